#!/usr/bin/env python3
"""Benchmark: the OpenWebRX IQ hot path on MI355X (BASELINE.json metric).

Workload (N=1, default `--config c3`, BASELINE config 3 = the north_star target on one GPU):
10 Msps synthetic cf32 IQ -> 16384-bin waterfall (FftChain: fps 9, v-overlap 0.3 -> avg 97,
hop 11454, ADPCM rows) + 256 client chains (86 NFM + 85 USB + 85 CW ClientDemodulatorChain:
Shift -> FirDecimate(833, 22223 taps) -> FractionalDecimator -> Bandpass -> Squelch -> demod ->
Agc -> Convert -> AdpcmEncoder(sync)).  `--config c2|c4|c5` runs the other BASELINE shapes per
GPU (32 NFM/AM chains; 61.44 Msps with a 65536-bin waterfall and 128 chains; 64 USB chains with
NoiseFilter).
A step is `--blocks-per-step` (4) blocks of `--block` IQ samples (2^20, SURVEY.md 8d: the driver's
20 steps stream 2^26.3 samples in 2^20-sample blocks) pushed through all of it, inputs resident
in HBM, outputs (waterfall rows, ADPCM audio, s-meter) copied back to host rings and drained
once per step.  The waterfall FFT launches once per `--wf-batch` frames (owrx_waterfall_
set_batch; eight per stream-A CU by default), not once per block.

N>1 (torchrun, one rank per GPU): rank 0 owns the stream and broadcasts each block over RCCL
(the path's one exchange step); every rank runs its own chains (weak scaling:
per-GPU work fixed), rank 0 also the waterfall.  value = the ingested stream's Msps (one stream
at any N); chains_total and chain_msamples_per_s give the aggregate chain work.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "IQ Msamples/s ingested + concurrent demod chains @ real-time, 1/2/4/8 GPU"
# BASELINE.json configs (per GPU): sample rate, waterfall bins, chains, chain modes, NoiseFilter
CONFIGS = {
    "c2": dict(fs=10000000, n_fft=16384, chains=32, modes=("nfm", "am"), nr=False,
               label="C2: 10 Msps cf32 IQ -> 16384-bin waterfall + %d NFM/AM chains per GPU"),
    "c3": dict(fs=10000000, n_fft=16384, chains=256, modes=("nfm", "usb", "cw"), nr=False,
               label="C3: 10 Msps cf32 IQ -> 16384-bin waterfall + %d NFM/USB/CW chains per GPU"),
    "c4": dict(fs=61440000, n_fft=65536, chains=128, modes=("nfm", "am", "usb", "cw"), nr=False,
               label="C4 (per GPU of 8): 61.44 Msps cf32 IQ -> 65536-bin waterfall + %d mixed "
                     "chains per GPU"),
    "c5": dict(fs=10000000, n_fft=16384, chains=64, modes=("usb",), nr=True,
               label="C5: 10 Msps cf32 IQ -> 16384-bin waterfall + %d USB chains with "
                     "NoiseFilter(10) per GPU"),
}
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: peak FP32 vector
HBM_PEAK_GBS = 8000.0
RIDGE = FP32_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)  # flop per byte where the roofs meet


def gen_stream_torch(torch, dev, fs, n, modes, offsets, seed=20251114):
    """Same signal model as openwebrx_amd.synth (AWGN 0.01 + one carrier per chain), generated on
    the GPU by the library's synthetic source (owrx_synth_iq: one kernel per 2^24 samples; bench
    data only)."""
    from openwebrx_amd import _lib
    out = torch.empty(n, dtype=torch.complex64, device=dev)
    code = {"nfm": 0, "am": 1, "usb": 2, "cw": 3, "lsb": 4}
    offs = np.asarray(offsets, np.float64)
    mds = np.asarray([code[m] for m in modes], np.int32)
    _lib.check(_lib.lib.owrx_synth_iq(dev.index or 0, out.data_ptr(), n, 0, float(fs), len(mds),
                                      offs.ctypes.data, mds.ctypes.data, seed, 0.01, 0.05),
               "owrx_synth_iq")
    return out


def _host_cpu():
    """nproc, the CPU model, the cores this process may use (affinity) and the cgroup CPU quota."""
    info = {"nproc": os.cpu_count()}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = info["nproc"]
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    info["cgroup_quota_cpus"] = quota
    return info


def _log(msg):
    """progress on stderr (a long run must keep writing: gpurun takes 180 s of silence as a hang)"""
    print("[bench %.1fs] %s" % (time.perf_counter() - _T0, msg), file=sys.stderr, flush=True)


_T0 = time.perf_counter()


def cpu_baseline(fs, n_fft, hop, avg, plist):
    """The CPU baseline: oracle/cpu_baseline.c -- the same
    waterfall + chains with the costly stages in fp32 / AVX2-FMA like csdr (Shift + FirDecimate,
    waterfall FFT), the 12 kHz tail from the oracle -- timed on this host: once on 1 core and once
    on every core this process may use (the cgroup quota if one is set, else the affinity set).
    `value` is the all-cores rate.  Also: the waterfall alone (csdr runs it as one thread:
    FftChain's modules are one pipe), and the largest chain count the host keeps real time with
    at this stream rate -- predicted from the 1-core per-chain and waterfall costs on the
    available cores, then checked on 2 s of stream (stepped down until it keeps up)."""
    import ctypes
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    from openwebrx_amd import synth
    host = _host_cpu()
    allc = host["affinity"]
    if host["cgroup_quota_cpus"]:
        allc = max(1, min(allc, int(host["cgroup_quota_cpus"])))
    lib = orc.lib()
    fn = lib.cpb_run_workload
    fn.restype = ctypes.c_int64
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_float, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    cps = [orc.chain_from_engine_params(p) for p in plist]
    iq_cache = {}

    def timed(n, threads, nchains):
        if n not in iq_cache:
            iq_cache.clear()
            iq_cache[n] = synth.make_iq(fs, n, ["nfm"])[0]
        arr = (orc.ChainParams * max(1, nchains))(*[cps[c % len(cps)] for c in range(max(1, nchains))])
        t0 = time.perf_counter()
        fn(iq_cache[n].ctypes.data, n, n_fft, hop, avg, -70.0, arr, nchains, threads)
        return time.perf_counter() - t0

    # sized for a few seconds each: 2^21 samples on one core, 2^22 x cores/8 on all of them
    n1 = 1 << 21
    dt1 = timed(n1, 1, len(cps))
    nall = max(n1, (1 << 22) * max(1, allc) // 8)
    dta = timed(nall, allc, len(cps))
    _log("cpu baseline: waterfall only")
    nw = 1 << 22
    dtw = timed(nw, 1, 0)
    t_w = dtw / nw                                    # core-seconds per sample, waterfall
    t_c = max(1e-15, (dt1 / n1 - t_w) / len(cps))     # core-seconds per sample and chain
    if t_w * fs >= 1.0:
        c_pred = 0
    else:
        c_pred = max(0, int((allc / fs - t_w) / t_c))
    checks = []
    nv = int(2 * fs)
    c_try = c_pred
    c_ok = 0
    for _ in range(4):
        if c_try <= 0:
            break
        _log("cpu baseline: real-time check with %d chains" % c_try)
        dtv = timed(nv, allc, c_try)
        checks.append({"chains": c_try, "stream_seconds": round(nv / fs, 2), "wall_s": round(dtv, 2)})
        if dtv <= nv / fs:
            c_ok = c_try
            break
        c_try = int(c_try * 0.85)
    # the csdr-shaped leg: one thread per module per chain, bounded queues between
    # modules (oracle/cpu_baseline.c cpb_run_pipeline), the OS scheduling them on this process's
    # cores; a bounded sample of the same workload
    _log("cpu baseline: csdr-shaped (thread per module per chain)")
    fp = lib.cpb_run_pipeline
    fp.restype = ctypes.c_int64
    fp.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_float, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    npipe = 1 << 22
    if npipe not in iq_cache:
        iq_cache.clear()
        iq_cache[npipe] = synth.make_iq(fs, npipe, ["nfm"])[0]
    arr = (orc.ChainParams * len(cps))(*cps)
    nth = ctypes.c_int(0)
    t0 = time.perf_counter()
    rb = fp(iq_cache[npipe].ctypes.data, npipe, n_fft, hop, avg, -70.0, arr, len(cps), ctypes.byref(nth))
    dtp = time.perf_counter() - t0
    csdr_shaped = {"value": round(npipe / dtp / 1e6, 3), "unit": "Msps", "cores": allc,
                   "threads": int(nth.value), "output_bytes": int(rb),
                   "sample": "%d samples (%.2f s of stream) through the waterfall + %d chains, one "
                             "thread per module (%d threads) with bounded chunk queues between "
                             "modules, %.2f s wall on %d cores; chunk-local module state (a timing "
                             "model, not the exact stream)" % (npipe, npipe / fs, len(cps),
                                                               nth.value, dtp, allc)}
    return {"value": round(nall / dta / 1e6, 3), "unit": "Msps", "cores": allc,
            "kind": "port",
            "csdr_shaped": csdr_shaped,
            "one_core_msps": round(n1 / dt1 / 1e6, 4),
            "waterfall_only_msps": round(nw / dtw / 1e6, 3),
            "waterfall_only_cores": 1,
            "max_realtime_chains": c_ok,
            "max_realtime_chains_predicted": c_pred,
            "max_realtime_chains_checks": checks,
            "host": host,
            "sample": "%d samples (%.2f s of %.2f Msps IQ) through the waterfall + %d chains on %d "
                      "cores, %.2f s wall (1 core: %d samples, %.2f s); waterfall alone: %d samples "
                      "on 1 core, %.2f s; oracle/cpu_baseline.c (fp32, AVX2+FMA, OpenMP over chains)"
                      % (nall, nall / fs, fs / 1e6, len(plist), allc, dta, n1, dt1, nw, dtw)}


def realtime_check(Engine, params, fs, n_fft, hop, avg, plist, stream_host, seconds, block,
                   ddc_mode="fast", churn=False, pipelined=None, wf_batch=0, wf_cap_ms=0.0):
    """SURVEY.md 8d measurement 1: feed the stream at its nominal rate through the host push path
    (SDR -> host cf32 -> PCIe -> HBM, owrx_push_iq) to a fresh engine with the same waterfall and
    chains; every block is pushed on its wall-clock deadline.  Without `churn` each block is then
    synced and drained (latency = push to outputs in the host rings).  Keeps up when no output
    ring overran and every block finished within its own period.

    `pipelined` (default: with churn) runs the loop like a live server instead: no per-block sync (outputs are read as
    they arrive, the pipeline keeps up to four blocks in flight); with `churn`, right after each
    push one client leaves, another joins (owrx_chain_destroy + owrx_chain_create) and a third drags its
    bandpass (owrx_chain_set_bandpass) while that block and its predecessors are in flight.  It
    keeps up when every push returned before the next deadline (a GPU slower than the stream
    back-pressures push) and nothing overran; `pipeline_drains` counts full pipeline drains inside
    the loop (none: those calls do not drain); the host latency of each call is reported.

    `wf_batch` > 1: the waterfall batches its FFT launches as the headline engine does
    (owrx_waterfall_set_batch), bounded by `wf_cap_ms` of wall clock (owrx_waterfall_set_latency);
    the rows' measured latency (the call of the block that completed a row to the row in the
    host ring) is reported."""
    if pipelined is None:
        pipelined = churn
    t_setup = time.perf_counter()
    hist = (wf_batch + 16) * hop + 2 * n_fft + block if wf_batch > 1 else 0
    eng = Engine(fs, max_block=block, history=hist)
    eng.set_ddc_mode(ddc_mode)
    wf = eng.waterfall(n_fft, hop, avg, adpcm=True)
    if wf_batch > 1:
        wf.set_batch(wf_batch)
        if wf_cap_ms > 0:
            wf.set_latency(wf_cap_ms)
    chains = []
    try:
        for i, p in enumerate(plist):
            chains.append(eng.chain(p))
            if i % 4096 == 4095:
                _log("  %d chains created" % (i + 1))
        eng.sync()
    except Exception:  # e.g. out of device memory: give it back before the caller goes on
        eng.close()
        raise
    t_setup = time.perf_counter() - t_setup
    period = block / fs
    nblocks = max(1, int(seconds / period))
    lat, joins, leaves, bps = [], [], [], []
    wf_settings = [(avg, hop), params.fft_parameters(fs, n_fft, 25, 0.3)]
    wf_every = max(1, int(round(1.0 / period)))  # blocks per second of stream
    wf_alt, wf_set_ms = 0, []
    tp = ts = tr = 0.0  # host seconds in push (block build + launches), sync, output reads
    st0 = eng.stats()
    rng = np.random.default_rng(7)
    # the harness's own Python objects (C chain handles and parameter records) make the
    # collector's full passes take tens of ms at 10^5 chains: none during the paced loop
    import gc
    gc_was = gc.isenabled()
    gc.collect()
    gc.disable()
    parts = []  # per block: (push, reads) seconds
    hk = ("host_ms_wait_slots", "host_ms_collect", "host_ms_drain_wait", "host_ms_drain_copy",
          "host_ms_wait_input", "host_ms_build", "host_ms_launch", "pipeline_drains", "pool_allocs")
    hparts = []  # per block: the engine's own host-time deltas (hk) over push + reads
    handles = eng.handles(chains)  # kept in step with `chains` (read_chains takes the array)
    t0 = time.perf_counter()
    for i in range(nblocks):
        deadline = t0 + i * period
        wait = deadline - time.perf_counter()
        if wait > 0:
            time.sleep(wait)
        sa = eng.stats()
        a = time.perf_counter()
        eng.push(stream_host[(i * block) % (stream_host.size - block):][:block])
        b = time.perf_counter()
        tp += b - a
        if churn and i % wf_every == wf_every - 1:
            # the client's waterfall settings change once a second (fps 9 <-> 25, the
            # SpectrumThread's setProperty path, owrx/fft.py:49-56): no drain
            wf_alt = 1 - wf_alt
            a_, h_ = wf_settings[wf_alt]
            w0 = time.perf_counter()
            wf.set(h_, a_, True)
            wf_set_ms.append(time.perf_counter() - w0)
        if churn and chains:
            c0 = time.perf_counter()
            j = int(rng.integers(len(chains)))
            chains.pop(j).close()
            c1 = time.perf_counter()
            chains.append(eng.chain(plist[int(rng.integers(len(plist)))]))
            c2 = time.perf_counter()
            handles[j:-1] = handles[j + 1:].copy()
            handles[-1] = chains[-1].id
            k = int(rng.integers(len(chains)))
            lo = float(rng.uniform(-0.2, 0.0))
            chains[k].set_bandpass(params.f32(lo), params.f32(lo + 0.15))
            c3 = time.perf_counter()
            leaves.append(c1 - c0)
            joins.append(c2 - c1)
            bps.append(c3 - c2)
        c = time.perf_counter()
        if not pipelined:
            eng.sync()
        d = time.perf_counter()
        eng.read_chains(handles)
        wf.read()
        e = time.perf_counter()
        sb = eng.stats()
        hparts.append([round(sb[k] - sa[k], 1) for k in hk])
        ts += d - c
        tr += e - d
        # pipelined: how late the block's push (and this iteration) ran against its deadline
        lat.append(e - a if not pipelined else e - deadline)
        parts.append((b - a, e - d))
    st_loop = eng.stats()
    if gc_was:
        gc.enable()
    eng.sync()
    # pipelined: the level's last outputs are in the host rings within one period of its last
    # deadline (a GPU slower than the stream accumulates lag block by block)
    finish_lag = time.perf_counter() - (t0 + nblocks * period)
    st = eng.stats()
    host = {"push_ms": round(1e3 * tp / nblocks, 3), "sync_ms": round(1e3 * ts / nblocks, 3),
            "read_ms": round(1e3 * tr / nblocks, 3)}
    for k in ("host_ms_process", "host_ms_wait_input", "host_ms_wait_slots", "host_ms_wait_rows"):
        host[k] = round((st[k] - st0[k]) / nblocks, 3)
    nrow = st["wf_rows_latency_n"] - st0["wf_rows_latency_n"]
    rows = {"rows": int(st["waterfall_rows"] - st0["waterfall_rows"]),
            "batch_frames": wf_batch, "cap_ms": wf_cap_ms,
            "latency_ms_max": round(st["wf_row_latency_ms_max"], 3),
            "latency_ms_mean": round((st["wf_row_latency_ms_sum"] - st0["wf_row_latency_ms_sum"])
                                     / max(1, nrow), 3),
            "launches": int(st["waterfall_launches"] - st0["waterfall_launches"])}
    eng.close()
    extra = {}

    def summ(v):
        return {"mean": round(1e3 * sum(v) / len(v), 3), "max": round(1e3 * max(v), 3), "n": len(v)}
    if joins:
        extra = {"client_join_ms": summ(joins), "client_leave_ms": summ(leaves),
                 "set_bandpass_ms": summ(bps),
                 "waterfall_fps_changes": len(wf_set_ms),
                 "waterfall_set_ms": summ(wf_set_ms) if wf_set_ms else None,
                 "pipeline_drains": int(st_loop["pipeline_drains"] - st0["pipeline_drains"])}
    return {**extra, "seconds": round(nblocks * period, 2), "stream_msps": fs / 1e6, "chains": len(plist),
            "setup_s": round(t_setup, 2),
            "blocks": nblocks, "block_period_ms": round(1e3 * period, 2),
            "max_block_latency_ms": round(1e3 * max(lat), 3),
            "mean_block_latency_ms": round(1e3 * sum(lat) / len(lat), 3),
            # the five latest blocks: [block index, latency, push, reads] in ms, and the
            # engine's host time in them (worst_blocks_host: hk's deltas over push + reads)
            "worst_blocks": [[i, round(1e3 * lat[i], 1), round(1e3 * parts[i][0], 1),
                              round(1e3 * parts[i][1], 1)]
                             for i in sorted(range(len(lat)), key=lambda i: -lat[i])[:5]],
            "worst_blocks_host": {"fields": list(hk),
                                  "blocks": {str(i): hparts[i] for i in
                                             sorted(range(len(lat)), key=lambda i: -lat[i])[:5]}},
            "latency_ms_p99": round(1e3 * float(np.percentile(lat, 99)), 3),
            "latency_definition": ("push start to outputs in the host rings (sync per block)"
                                   if not pipelined else
                                   "deadline to the end of the block's push + churn + reads "
                                   "(pipelined, no per-block sync)"),
            "overruns": int(st["overruns"]),
            "waterfall_rows": rows,
            "host_per_block": host,
            "finish_lag_ms": round(1e3 * finish_lag, 3) if pipelined else None,
            "keeps_up": bool(st["overruns"] == 0 and max(lat) < period and
                             (not pipelined or finish_lag < period)),
            "path": "host cf32 -> owrx_push_iq (PCIe) -> engine"}


def max_realtime_chains(Engine, params, fs, n_fft, hop, avg, modes, offsets_of, stream_host,
                        seconds, block, ladder, ddc_mode, budget_s, agree=None, world=1,
                        hold_s=0.0, wf_batch=0, wf_cap_ms=0.0):
    """BASELINE.md 3 / SURVEY.md 8d: the largest chain count C (from `ladder`) for which the paced
    real-time check at the config's stream rate keeps up (no overrun, every block within its
    period), with the waterfall running too.  Stops at the first failure (a level that does not
    keep up, or cannot even be set up, e.g. out of device memory) or when the next level would
    exceed the time budget.  At N>1 every rank runs each level at the same time on its own GPU
    (C chains each, the stream pushed to every rank); a level passes when every rank kept up
    (`agree` reduces over ranks), and the job's figure is C x N."""
    agree = agree or (lambda v, op: v)
    levels, best = [], 0
    t0 = time.perf_counter()
    for C in ladder:
        elapsed = agree(time.perf_counter() - t0, "max")
        if levels and elapsed + 2.5 * levels[-1].get("setup_s", 0) + seconds > budget_s:
            levels.append({"chains": C, "skipped": "time budget"})
            break
        ms = [modes[c % len(modes)] for c in range(C)]
        plist = [params.chain_params(fs, o, m) for o, m in zip(offsets_of(C), ms)]
        _log("capacity level: %d chains" % C)
        try:
            r = realtime_check(Engine, params, fs, n_fft, hop, avg, plist, stream_host, seconds,
                               block, ddc_mode, pipelined=True, wf_batch=wf_batch,
                               wf_cap_ms=wf_cap_ms)
            ok = r["keeps_up"]
        except Exception as exc:  # e.g. out of device memory: this level does not run
            r, ok = {"chains": C, "error": str(exc)[:200], "setup_s": 0.0}, False
            _log("  failed: %s" % exc)
        ok = bool(agree(1.0 if ok else 0.0, "min") > 0)
        lvl = {k: r[k] for k in ("chains", "max_block_latency_ms", "mean_block_latency_ms",
                                 "finish_lag_ms", "overruns", "setup_s", "host_per_block",
                                 "waterfall_rows", "worst_blocks", "worst_blocks_host", "error")
               if k in r}
        lvl["keeps_up"] = ok
        if world > 1:
            lvl["max_block_latency_ms_all_ranks"] = round(agree(r.get("max_block_latency_ms", 1e9), "max"), 3)
        levels.append(lvl)
        if "error" not in r:
            _log("  setup %.2f s, keeps_up %s, max block latency %.2f ms, finish lag %.2f ms, "
                 "overruns %d, host/block %s" % (r["setup_s"], ok, r["max_block_latency_ms"],
                                                 r["finish_lag_ms"], r["overruns"],
                                                 json.dumps(r["host_per_block"])))
        if not ok:
            break
        best = C
    failing = next((l["chains"] for l in levels if l.get("keeps_up") is False), None)
    holds, held = [], 0
    passed = [l["chains"] for l in levels if l.get("keeps_up")]
    if best and hold_s > 0:
        # the top passing level once more, held for hold_s of stream (60 s); if
        # it does not keep up that long, the passing levels below it in turn, at most three
        # holds in all (one slow block of 572 fails a hold: round 5's driver-form run failed it
        # at 196 608 and 131 072 chains, each on one 140-440 ms block)
        import gc
        for C in passed[::-1][:3]:
            gc.collect()  # the failed level's Python objects (its engine is closed already)
            _log("capacity hold: %d chains for %.0f s" % (C, hold_s))
            ms = [modes[c % len(modes)] for c in range(C)]
            plist = [params.chain_params(fs, o, m) for o, m in zip(offsets_of(C), ms)]
            try:
                r = realtime_check(Engine, params, fs, n_fft, hop, avg, plist, stream_host,
                                   hold_s, block, ddc_mode, pipelined=True, wf_batch=wf_batch,
                                   wf_cap_ms=wf_cap_ms)
                ok = bool(agree(1.0 if r["keeps_up"] else 0.0, "min") > 0)
                h = {k: r[k] for k in ("chains", "seconds", "blocks", "max_block_latency_ms",
                                       "mean_block_latency_ms", "latency_ms_p99", "finish_lag_ms",
                                       "overruns", "waterfall_rows", "host_per_block",
                                       "worst_blocks", "worst_blocks_host") if k in r}
                h["keeps_up"] = ok
            except Exception as exc:
                h = {"chains": C, "error": str(exc)[:200], "keeps_up": False}
            _log("  hold: " + json.dumps(h))
            holds.append(h)
            if h["keeps_up"]:
                held = C
                break
    return {"max_realtime_chains": best * world, "per_gpu": best, "first_failing_level": failing,
            "max_realtime_chains_held": held * world, "hold_seconds": hold_s, "holds": holds,
            "stream_msps": fs / 1e6, "block_samples": block,
            "seconds_per_level": seconds, "levels": levels,
            "waterfall": "batched launches of up to %d frames, bounded by %.0f ms of wall clock "
                         "(owrx_waterfall_set_batch + owrx_waterfall_set_latency)"
                         % (wf_batch, wf_cap_ms) if wf_batch > 1 else "per-block launches",
            "note": "paced pushes of host cf32 through owrx_push_iq at the stream's wall-clock rate, "
                    "waterfall + C chains per GPU (modes cycled), pipelined like a server (outputs "
                    "read as they arrive, no per-block sync: a push that cannot keep its deadline "
                    "fails the level); largest C "
                    "that kept up on every GPU, times N; the ladder stops at the first level that did "
                    "not (first_failing_level) or the time budget"}


def _scaled_steps(fs, n_fft):
    """The recorded NFM client graph (tests/golden/dsp_graph.json, 10 Msps) and FftChain graph
    (tests/golden/spectrum_graph.json) at another input rate: the Selector's FirDecimate /
    FractionalDecimator parameters from params.decimation (Decimator._getDecimation, golden-
    pinned by tests/test_params.py; no FractionalDecimator where the rate divides, as
    selector.py:32 builds none) and the FftChain's from params.fft_parameters; the rest of the
    graph (12 kHz Bandpass, Squelch, demodulator, ClientAudioChain) is rate independent."""
    import copy
    import dsp_replay
    from openwebrx_amd import params
    s = copy.deepcopy(dsp_replay.steps()["nfm"])
    d, frac, tbw, cutoff = params.decimation(fs, 12000)
    keep, remap = [], {}
    for i, g, src in s["graph"]:
        if g["class"] == "FractionalDecimator" and frac == 1.0:
            remap[i] = remap[src]  # its readers read its input
            continue
        remap[i] = len(keep)
        keep.append((i, g, src))
    graph = []
    for i, g, src in keep:
        if g["class"] == "FirDecimate":
            g.update(decimation=d, transition=tbw, cutoff=cutoff)
        if g["class"] == "FractionalDecimator":
            g["rate"] = frac
        graph.append([remap[i], g, remap[src] if src >= 0 else src])
    s["graph"] = graph
    avg, hop = params.fft_parameters(fs, n_fft, 9, 0.3)
    with open(os.path.join(ROOT, "tests", "golden", "spectrum_graph.json")) as f:
        sg = copy.deepcopy({x["step"]: x for x in json.load(f)}["start_adpcm"])
    for g in sg["graph"]:
        for k in ("size", "fft_size"):
            if k in g:
                g[k] = n_fft
        if "every_n_samples" in g:
            g["every_n_samples"] = hop
        if "avg_number" in g:
            g["avg_number"] = avg
    return s, sg


def _dropin_run(fs, C, blocks, paced, pump_limit, steps=None):
    """One drop-in run: C ClientDemodulatorChain graphs as the reference builds them
    (tests/golden/dsp_graph.json "nfm": Shift -> FirDecimate -> ... -> AdpcmEncoder, one Shift
    rate per client) plus the SpectrumThread's FftChain (tests/golden/spectrum_graph.json
    "start_adpcm") on one wideband pycsdr Buffer, each output read by its own pump thread
    (owrx/dsp.py:846-863, owrx/fft.py:73), the stream written in 2^18-sample writes (the shim
    driver's block).  The driver plans and creates its segments on the first writes; the
    measured writes start once every segment runs and the driver has caught up."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dsp_replay  # graph rebuilder (data from tests/golden; no reference code)
    from openwebrx_amd import params, synth
    from openwebrx_amd.pycsdr import _graph
    from openwebrx_amd.pycsdr import modules as M
    from openwebrx_amd.pycsdr.types import Format
    if 2 * C + 1 > pump_limit:
        raise ValueError("%d pump threads over the limit %d" % (2 * C + 1, pump_limit))
    s = steps[0] if steps else dsp_replay.steps()["nfm"]
    offs = synth.carrier_offsets(fs, C)
    wide = M.Buffer(Format.COMPLEX_FLOAT, size=1 << 23)
    pumps, got = [], {}

    def pump(name, buf):
        r = buf.getReader()
        got[name] = [0, None]

        def run():
            for data in iter(r.read, None):  # csdr.chain.Chain.pump(reader.read, write)
                got[name][0] += len(data)
                got[name][1] = time.perf_counter()
        t = threading.Thread(target=run, name="dsp_pump_" + name, daemon=True)
        t.start()
        pumps.append((r, t))

    def teardown():  # the clients leave: every module stopped (chain.stop()), pumps joined
        _graph.finish(wide)
        for m in allmods:
            stop = getattr(m, "stop", None)
            if stop is not None:
                stop()
        for r, t in pumps:
            r.stop()
        for r, t in pumps:
            t.join(5)

    cls = [d["class"] for _, d, _ in s["graph"]]
    allmods = []
    for c in range(C):
        _, mods, outs, power = dsp_replay.build(s, wide=wide)
        allmods += mods
        mods[0].setRate(params.shift_rate(offs[c], fs))
        for m in mods:  # the recorded Python consumer of the wideband buffer: not served here
            if isinstance(m, M.Reader):
                m.stop()
        pump("audio%d" % c, outs[cls.index("AdpcmEncoder")])
        pump("smeter%d" % c, power)
    if steps:
        sg = steps[1]
    else:
        with open(os.path.join(ROOT, "tests", "golden", "spectrum_graph.json")) as f:
            sg = {x["step"]: x for x in json.load(f)}["start_adpcm"]
    fmods = [dsp_replay._make(d) for d in sg["graph"]]
    allmods += fmods
    for a, b in zip(fmods, fmods[1:]):
        buf = M.Buffer(a.getOutputFormat())
        a.setWriter(buf)
        b.setReader(buf.getReader())
    rows = M.Buffer(Format.CHAR)
    fmods[-1].setWriter(rows)
    fmods[0].setReader(wide.getReader())
    pump("waterfall", rows)

    blk = _graph.BLOCK
    iq, _ = synth.make_iq(fs, 8 * blk, ["nfm"] * 16)
    chunks = [iq[k * blk:(k + 1) * blk].tobytes() for k in range(8)]
    # set-up: a few writes make the driver plan and create every segment; wait until it runs
    # them all and has consumed what it was given
    t_setup = time.perf_counter()
    drv = None
    for k in range(4):
        wide.write(chunks[k % 8])
        drv = drv or _graph._drivers.get(id(wide))
    t_log = t_setup
    while time.perf_counter() - t_setup < 60:
        drv = drv or _graph._drivers.get(id(wide))
        if drv and drv.state != "RUNNING":
            break
        if drv and drv.engine is not None and len(drv.segments) == C + 1 \
                and drv.reader.available() == 0:
            break
        if time.perf_counter() - t_log > 5:
            t_log = time.perf_counter()
            _log("  setup: driver %s, segments %d" % (drv and drv.state,
                                                      len(drv.segments) if drv else 0))
        time.sleep(0.01)
    fused = bool(drv and drv.engine is not None and len(drv.segments) == C + 1)
    t_setup = time.perf_counter() - t_setup
    if not fused:
        state = (drv.state, str(drv.error)[:160]) if drv else ("no driver", "")
        teardown()
        raise RuntimeError("drop-in did not fuse %d clients in %.0f s: %s" % (C, t_setup, state))
    a0 = sum(v[0] for v in got.values())
    lag, t0 = [], time.perf_counter()
    period = blk / fs
    for k in range(blocks):
        if paced:
            wait = t0 + k * period - time.perf_counter()
            if wait > 0:
                time.sleep(wait)
        else:  # as fast as the driver takes it: at most four writes ahead of it
            while drv.reader.available() > 4 * 8 * blk:
                time.sleep(0.0002)
        wide.write(chunks[k % 8])
        lag.append(drv.reader.available() / 8 / blk)
    t_last = time.perf_counter()
    while drv.reader.available() > 0 and time.perf_counter() - t_last < 30:
        time.sleep(0.002)
    t_fed = time.perf_counter()
    time.sleep(period)  # the last block's outputs: a period for the pumps to receive them
    last = max(v[1] or 0 for v in got.values())
    audio = [got["audio%d" % c][0] for c in range(C)]
    out_bytes = sum(v[0] for v in got.values()) - a0
    wf_bytes = got["waterfall"][0]
    teardown()
    t_end = max(t_fed, last)
    res = {"clients": C, "pump_threads": len(pumps), "fused": fused,
           "setup_s": round(t_setup, 2), "writes": blocks, "write_samples": blk,
           "max_driver_lag_blocks": round(max(lag), 2),
           "mean_driver_lag_blocks": round(sum(lag) / len(lag), 3),
           "audio_bytes_min": min(audio), "waterfall_bytes": wf_bytes,
           "output_bytes": out_bytes}
    if paced:
        finish_lag = t_end - t_last
        res["finish_lag_ms"] = round(1e3 * finish_lag, 1)
        res["period_ms"] = round(1e3 * period, 1)
        res["keeps_up"] = bool(fused and max(lag) <= 2.0 and finish_lag < period + 0.05
                               and min(audio) > 0)
    else:
        res["msps"] = round(blocks * blk / (t_end - t0) / 1e6, 2)
        res["seconds"] = round(t_end - t0, 3)
    return res


def dropin_c4(clients, seconds, pump_limit):
    """The drop-in at C4's rate on one GPU: 61.44 Msps into the 65 536-bin
    FftChain plus `clients` NFM ClientDemodulatorChain graphs (the recorded graphs at that rate,
    _scaled_steps), paced at the stream's wall-clock rate, every output on its own pump."""
    fs = 61440000
    _log("drop-in C4: %d clients paced at 61.44 Msps" % clients)
    from openwebrx_amd.pycsdr import _graph
    blk = _graph.BLOCK
    try:
        r = _dropin_run(fs, clients, max(8, int(seconds * fs / blk)), True, pump_limit,
                        steps=_scaled_steps(fs, 65536))
    except Exception as exc:
        r = {"clients": clients, "error": str(exc)[:200], "keeps_up": False}
    r["stream_msps"] = fs / 1e6
    r["fft_size"] = 65536
    _log("  " + json.dumps(r))
    return r


def dropin_check(fs, clients, ladder, seconds, budget_s, pump_limit):
    """what the drop-in (pycsdr shim -> _graph.EngineDriver -> engine) runs.
    `msps`: the shim path's ingest rate with `clients` clients, the stream written as fast as the
    driver takes it; `max_clients`: the largest client count of `ladder` whose paced 10 Msps run
    keeps up (driver never more than two blocks behind the writer, every output delivered within
    a period of the last write), each output on its own pump thread."""
    import threading
    from openwebrx_amd.pycsdr import _graph
    blk = _graph.BLOCK
    t0 = time.perf_counter()
    _log("drop-in: %d clients unpaced (threads alive: %d)" % (clients, threading.active_count()))
    try:
        thr = _dropin_run(fs, clients, max(8, int(seconds * fs / blk)), False, pump_limit)
    except Exception as exc:
        thr = {"clients": clients, "error": str(exc)[:200]}
    levels, best = [], 0
    for C in ladder:
        if levels and time.perf_counter() - t0 + 2.5 * levels[-1].get("setup_s", 0) + seconds \
                > budget_s:
            levels.append({"clients": C, "skipped": "time budget"})
            break
        _log("drop-in: %d clients paced (threads alive: %d)" % (C, threading.active_count()))
        try:
            r = _dropin_run(fs, C, max(8, int(seconds * fs / blk)), True, pump_limit)
        except Exception as exc:
            r = {"clients": C, "error": str(exc)[:200], "keeps_up": False}
        levels.append(r)
        _log("  " + json.dumps(r))
        if not r["keeps_up"]:
            break
        best = C
    return {"msps": thr.get("msps"), "msps_clients": clients, "unpaced": thr,
            "max_clients_paced": best, "levels": levels,
            "stream_msps": fs / 1e6,
            "wf_latency_cap_ms": _graph.wf_latency_ms(),
            "note": "the pycsdr shim as the reference drives it: ClientDemodulatorChain graphs "
                    "(tests/golden/dsp_graph.json nfm) + the FftChain on one wideband Buffer, "
                    "fused by openwebrx_amd.pycsdr._graph onto one engine (2^18-sample blocks, "
                    "waterfall batched under the wall-clock row-latency cap), every output on "
                    "its own Python pump thread; msps = samples written / (first measured write "
                    "to the last output delivered); the ladder is bounded by %d pump threads "
                    "(the GPU box's task limit)" % pump_limit}


def pmc_traffic(prefix, config):
    """HBM bytes per launch of a kernel from the newest committed PMC summary OF THIS CONFIG
    (profiles/*_pmc_traffic_<config>.json, written by tools/pmc_traffic.py from rocprofv3 --pmc
    passes of this same bench command); (None, reason) when absent."""
    import glob
    import re

    def order(f):  # tags rNN<suffix>: round, then suffix a..z, then aa..zz (later in a round)
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic_%s.json" % config)),
                   key=order)
    if not files:
        return None, "no PMC summary committed for config %s" % config
    d = json.load(open(files[-1]))
    for k, v in d["kernels"].items():
        if k.startswith(prefix):
            return v["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)
    return None, "kernel absent from " + os.path.relpath(files[-1], ROOT)


def extra_block_run(Engine, fs, n_fft, hop, avg, wf_batch, plist, stream, total, xb, no_wf,
                    warm=3, timed=16):
    """The same workload on a fresh engine at `xb`-sample blocks (16 timed after 3 untimed),
    from the same resident recording: the block granularity's effect on the rate."""
    hist = (wf_batch + 16) * hop + 2 * n_fft + xb if wf_batch > 1 else 0
    eng = Engine(fs, max_block=xb, history=hist)
    eng.set_input_retention(8)
    eng.set_pipeline_depth(16)
    h = eng.history
    if h + (warm + timed) * xb > stream.numel():
        eng.close()
        return None
    wf = None
    if not no_wf:
        wf = eng.waterfall(n_fft, hop, avg, adpcm=True)
        if wf_batch > 1:
            wf.set_batch(wf_batch)
    chains = [eng.chain(p) for p in plist]
    base = stream.data_ptr() + 8 * h

    def one(i):
        eng.process_device(base + 8 * i * xb, xb)
        eng.read_chains(chains)
        if wf is not None:
            wf.read()
    for i in range(warm):
        one(i)
    eng.sync()
    t0 = time.perf_counter()
    for i in range(warm, warm + timed):
        one(i)
    eng.sync()
    dt = time.perf_counter() - t0
    eng.close()
    return {"block_samples": xb, "blocks": timed, "msps": round(timed * xb / dt / 1e6, 2),
            "ms_per_block": round(dt * 1e3 / timed, 3),
            "note": "a fresh engine (16 blocks in flight, retention 8) on the same recording, %d "
                    "untimed then %d timed blocks, outputs drained per block, final sync inside "
                    "the timed region" % (warm, timed)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--blocks-per-step", type=int, default=4,
                    help="blocks of --block samples per timed step (SURVEY.md 8d: throughput runs "
                         "2^26 samples streamed in 2^20-sample blocks; the driver's 20 steps x 4 "
                         "blocks = 2^26.3 samples, so the pipeline's end-of-run drain is not a "
                         "fifth of the run)")
    ap.add_argument("--extra-block", type=int, default=1 << 22,
                    help="a second, shorter run at this block size reported beside the headline "
                         "(block_2p22: the round-2 headline granularity; 0 = skip)")
    ap.add_argument("--block", type=int, default=1 << 20,
                    help="IQ samples per step (SURVEY.md 8d: 2^20-sample blocks)")
    ap.add_argument("--wf-batch", type=int, default=-1,
                    help="waterfall frames per FFT launch (owrx_waterfall_set_batch; -1: eight per "
                         "stream-A CU at N <= 16384, two above, 0: every block's frames in that "
                         "block)")
    ap.add_argument("--chains", type=int, default=None,
                    help="chains per GPU (default: the config's)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS),
                    help="BASELINE.json config shape (c3, the largest single-GPU config, is the "
                         "metric's; the others are reported for reference)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-waterfall", action="store_true")
    ap.add_argument("--no-pairing", action="store_true",
                    help="one engine block per 2^20-sample block (owrx_set_block_pairing off)")
    ap.add_argument("--block-group", type=int, default=int(os.environ.get("OWRX_BENCH_GROUP", "4")),
                    help="contiguous 2^20-sample blocks per engine block (owrx_set_block_group: "
                         "2 = pairs, 4 = quads, the default: driver form 10 124-10 144 vs 9 761-9 838 "
                         "Msps in pairs, profiles/r06_group_ab.txt; input retention raised to "
                         "4 x this when lower)")
    ap.add_argument("--realtime-seconds", type=float, default=3.0,
                    help="paced real-time check at 10 Msps through the host push path (0: skip)")
    ap.add_argument("--no-timing", action="store_true",
                    help="skip the per-kernel HIP-event brackets (roofline fields become null)")
    ap.add_argument("--ddc", default="fast", choices=("fast", "direct"),
                    help="DDC form: fast-convolution filter bank (default) or direct polyphase FIR")
    ap.add_argument("--churn-chains", type=int, default=16384,
                    help="chains of the paced churn check (join + leave + setBandpass every "
                         "block, no per-block sync; 0: skip)")
    ap.add_argument("--capacity-ladder",
                    default="256,1024,4096,16384,32768,65536,98304,131072,196608,221184,262144",
                    help="chain counts tried by the max_realtime_chains sweep ('' = skip)")
    ap.add_argument("--capacity-seconds", type=float, default=2.0,
                    help="seconds of paced stream per sweep level")
    ap.add_argument("--capacity-hold-seconds", type=float, default=60.0,
                    help="the top passing level once more for this long (0: skip)")
    ap.add_argument("--wf-latency-ms", type=float, default=100.0,
                    help="wall-clock bound on a ready waterfall frame's wait for its batch "
                         "(owrx_waterfall_set_latency; one 9 fps row period less a margin for "
                         "the launch itself)")
    ap.add_argument("--dropin-clients", type=int, default=256,
                    help="clients of the drop-in's unpaced throughput run (0: skip the drop-in)")
    ap.add_argument("--dropin-ladder", default="256,384,448",
                    help="client counts of the drop-in's paced ladder (2 pump threads each)")
    ap.add_argument("--dropin-seconds", type=float, default=3.0)
    ap.add_argument("--dropin-c4-clients", type=int, default=128,
                    help="clients of the drop-in run at C4's rate (61.44 Msps, 65536-bin "
                         "FftChain, paced; 0: skip)")
    ap.add_argument("--loop-blocks", type=int, default=0,
                    help="A/B: the recording holds this many blocks and the stream loops over "
                         "them (0: one recording as long as the run)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # ranks beyond the visible GPUs share them (rehearsal on a small box; the driver's scaling
    # runs have one GPU per rank)
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("OWRX_DIST_BACKEND", "nccl"), rank=rank,
                                world_size=world)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from openwebrx_amd import Engine, params
    cfg = CONFIGS[args.config]
    fs = cfg["fs"]
    n_fft = cfg["n_fft"]
    avg, hop = params.fft_parameters(fs, n_fft, 9, 0.3)
    C = args.chains if args.chains is not None else cfg["chains"]
    modes = [cfg["modes"][c % len(cfg["modes"])] for c in range(C)]
    from openwebrx_amd.synth import carrier_offsets
    offs = carrier_offsets(fs, C)
    # the job's chains: C per GPU (weak scaling), copy r listening 37 Hz * r off the carriers
    # (different chains, identical cost), dealt to ranks within (D, taps, mode) groups
    from openwebrx_amd.multi import IqBroadcast, shard_chains
    everything = [(o + 37 * r, m) for r in range(world) for o, m in zip(offs, modes)]
    mine = shard_chains(everything, world, rank, key=lambda it: it[1])
    plist = [params.chain_params(fs, o, m, nr_enabled=cfg["nr"], nr_threshold=10)
             for o, m in mine]

    block = args.block
    # waterfall batching (rank 0 of a one-GPU run): the engine keeps enough history for the
    # batch's frames, and the FFT runs once per batch instead of once per block
    wf_batch = 0
    if rank == 0 and not args.no_waterfall:  # the waterfall runs on rank 0 at every N
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        # sixteen frames per stream-A CU for the 16384-point kernel (two groups of 8 per
        # workgroup: its start-up and first frame amortise over the frames, 0.294 vs 0.259 of
        # HBM at 8 per CU in the micro, profiles/r05_wf_micro.txt); two per CU above it (each
        # frame is 4 or 2 sub-frames of wf_fft_q16 after the DIF split).  The row-latency cap
        # bounds the wait at real-time rates.
        per_cu = 16 if n_fft <= 16384 else 2
        wf_batch = per_cu * max(1, cus - 16) if args.wf_batch < 0 else args.wf_batch
    history = (wf_batch + 16) * hop + 2 * n_fft + block if wf_batch > 1 else 0
    eng = Engine(fs, max_block=block, device=local, history=history)
    eng.set_ddc_mode(args.ddc)
    # the stream is a resident recording on rank 0 and a ring of broadcast windows on the other
    # ranks (IqBroadcast sizes its ring to the retention): every block stays valid for
    # `retention` further blocks, so the host may run that far ahead of stream A
    # (owrx_set_input_retention), at every N
    group = 1 if args.no_pairing else max(1, min(4, args.block_group))
    retention = int(os.environ.get("OWRX_BENCH_RETENTION", "8"))
    if group > 2:
        retention = max(retention, 4 * group)  # the host stays 3 engine blocks ahead (in_keep)
    eng.set_input_retention(retention)
    # 16 blocks in flight for the headline engine (256 chains: a few MB of staging per block);
    # the capacity ladder's engines keep the default 8 (their staging grows with the chains)
    depth = int(os.environ.get("OWRX_BENCH_DEPTH", "16"))
    eng.set_pipeline_depth(depth)
    # block pairing (owrx_set_block_pairing) on every rank: two 2^20-sample blocks per engine
    # launch sequence, the DDC GEMM reading the filter spectra once for both, outputs
    # byte-identical (test_block_pairing_same_outputs).  A pair must be contiguous in memory:
    # rank 0's recording is, and ranks > 0 receive each pair in one broadcast into one
    # [history | 2 blocks] window (IqBroadcast(pair=True), round 6), so every rank runs the N = 1
    # engine
    pairing = group > 1 and retention >= 2 * group
    if pairing:
        eng.set_block_group(group)
    hist = eng.history
    wf = None
    if rank == 0 and not args.no_waterfall:
        wf = eng.waterfall(n_fft, hop, avg, adpcm=True)
        # two whole rounds of the FFT launch where the engine deals it in rounds (16384 bins:
        # stream A's resident workgroups x 8 frames; no idle last round and no tail split,
        # profiles/r05_wf_tail_batch_ab.txt); the history above was sized for the larger default
        rnd = wf.round_frames()
        if wf_batch > 1 and args.wf_batch < 0 and rnd > 0 and 2 * rnd <= wf_batch:
            wf_batch = 2 * rnd
        if wf_batch > 1:
            wf.set_batch(wf_batch)
            wf.set_latency(args.wf_latency_ms)
    chains = [eng.chain(p) for p in plist]

    # engine priming before the W warmup steps: the first ~10 blocks of a fresh engine include
    # one-off host stalls of ~7 ms (first launches / queue setup on the four streams; measured at
    # global blocks 2-9 on MI355X), so at least 12 untimed blocks precede the timed region
    # whatever W is (12 in all); reported as "priming_blocks"
    bps = max(1, args.blocks_per_step)
    prime = max(0, -(-(12 - args.warmup * bps) // bps))  # priming steps: >= 12 untimed blocks
    nsteps = prime + args.warmup + args.steps
    total = nsteps * bps * block
    loop = args.loop_blocks if 0 < args.loop_blocks < nsteps * bps else 0
    span = loop * block if loop else total  # samples of the recording after the history
    stream = None
    if rank == 0:
        stream = gen_stream_torch(torch, dev, fs, hist + span, modes, offs)
        base = stream.data_ptr() + 8 * hist
    bcast = None
    if dist:
        # the broadcast windows carry the chains' history (the engine default on ranks > 0, the
        # same on every rank: the collectives must match); rank 0 keeps its own, longer
        # waterfall-batch history in front of the recording, so its view starts that much later
        t = torch.tensor([float(hist if rank else 0)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        hist_b = int(t.item())
        src_view = stream[hist - hist_b:] if rank == 0 else None
        bcast = IqBroadcast(torch, dist, dev, hist_b, block, stream=src_view, retention=retention,
                            group=group if pairing else 1)
    torch.cuda.synchronize(dev)

    def drain():
        # every chain's audio and s-meter values in two native calls (a one-thread server pump)
        audio, _, _, _ = eng.read_chains(chains)
        nbytes = int(audio.size)
        if wf is not None:
            nbytes += len(wf.read())
        return nbytes

    host_s = {"process": 0.0, "drain": 0.0, "process_t": 0.0, "drain_t": 0.0}

    def step(i, timed=False):
        t0 = time.perf_counter()
        n = _step(i)
        dt_ = time.perf_counter() - t0
        host_s["drain"] += dt_
        if timed:
            host_s["drain_t"] += dt_
        return n

    def _step(i):
        for j in range(i * bps, (i + 1) * bps):
            if world == 1:
                t0 = time.perf_counter()
                eng.process_device(base + 8 * (j % loop if loop else j) * block, block)
                dt_ = time.perf_counter() - t0
                host_s["process"] += dt_
                if call_log is not None and i >= prime + args.warmup and len(call_log) < 64:
                    call_log.append(("process", j, round(1e3 * dt_, 3)))
                if i >= prime + args.warmup:
                    host_s["process_t"] += dt_
            else:  # the one exchange step: rank 0's block to every rank over RCCL
                # block j + 1's broadcast is enqueued before block j is processed, so it runs
                # beside this block's host and GPU work (three windows, multi.IqBroadcast)
                if j + 1 < nsteps * bps:
                    bcast.issue(j + 1)
                t, off = bcast.wait(j)
                # stream A waits on the GPU for this broadcast (owrx_wait_stream on torch's
                # stream, which the collective's wait() ordered behind it): no host wait, the
                # engine's streams keep earlier blocks in flight
                if rank != 0:
                    eng.wait_stream(torch.cuda.current_stream(dev).cuda_stream)
                eng.process_device(t.data_ptr() + 8 * off, block)
        if call_log is not None and i >= prime + args.warmup and len(call_log) < 64:
            t1 = time.perf_counter()
            n = drain()
            call_log.append(("drain", i, round(1e3 * (time.perf_counter() - t1), 3)))
            return n
        return drain()

    # OWRX_BENCH_CALLS=1: the host time of each call of the first timed steps (diagnostic)
    call_log = [] if os.environ.get("OWRX_BENCH_CALLS") else None
    for i in range(prime + args.warmup):
        step(i)
    # the Python driver's garbage collector stalls the host for milliseconds at times; keep it
    # out of the timed region (the engine itself allocates nothing per block)
    import gc
    gc.collect()
    gc.disable()
    eng.sync()
    # the warm-up's last outputs (what the sync above completed: its held blocks, the pending
    # waterfall batch's rows) are read here, with the warm-up: left in the rings, the first timed
    # step's read took them (0.8 ms of host time, and the host launched the second timed engine
    # block that much later: stream C then idled ~0.6 ms).  OWRX_BENCH_PREDRAIN=0: the old order (A/B)
    if os.environ.get("OWRX_BENCH_PREDRAIN", "1") != "0":
        drain()
    # HIP events in every 8th block (each block's events cost host time: ~8 more API calls; the
    # waterfall's batched launches are all timed)
    eng.set_timing(not args.no_timing, every=8)
    s0 = eng.stats()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    out_bytes = 0
    marks = []
    for i in range(prime + args.warmup, nsteps):
        out_bytes += step(i, timed=True)
        marks.append(time.perf_counter() - t0)
    eng.sync()
    marks.append(time.perf_counter() - t0)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    s1 = eng.stats()
    xblock = None
    if world == 1 and args.extra_block and args.extra_block != block:
        xblock = extra_block_run(Engine, fs, n_fft, hop, avg, wf_batch, plist, stream, span,
                                 args.extra_block, args.no_waterfall)
    gc.enable()
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    print("host seconds over all steps: process_device %.4f, step total %.4f, wall %.4f"
          % (host_s["process"], host_s["drain"], dt), file=sys.stderr)
    print("step marks (ms): " + " ".join("%.2f" % (1e3 * m) for m in marks), file=sys.stderr)
    if call_log:
        print("first timed calls (ms): " + " ".join("%s%d:%.3f" % c for c in call_log), file=sys.stderr)
    samples = args.steps * bps * block
    value = samples / dt / 1e6  # the one ingested stream, at any N (chains scale with N)
    ms_step = dt * 1e3 / args.steps
    # DDC work: the fast-convolution GEMM (fc_mac) is the dominant kernel of the chain path;
    # achieved = its algorithmic flop per launch / its average launch time (HIP events on the
    # engine's stream A, around that kernel only)
    D, frac, tbw, cutoff = params.decimation(fs, 12000)
    T = int(4.0 / float(np.float32(tbw)))
    T += 1 - (T % 2)
    d = {k: s1[k] - s0[k] for k in s1}
    tsteps = max(1, d["timed_blocks"])  # the gpu_ms_* sums cover the timed blocks only
    # caller blocks per engine block (2 when every pair formed: owrx_set_block_pairing)
    per_engine = max(1.0, d["samples_in"] / block / max(1, d["blocks"]))
    # every rank's grouping (owrx_set_block_group over IqBroadcast(group=g) windows on ranks > 0):
    # the fewest caller blocks per engine block any rank formed
    per_engine_min = per_engine
    if dist:
        te = torch.tensor([per_engine], dtype=torch.float64, device=dev)
        dist.all_reduce(te, op=dist.ReduceOp.MIN)
        per_engine_min = float(te.item())
    tblocks = tsteps * per_engine
    launches = d["ddc_launches"]
    ddc_ms = d["gpu_ms_ddc"]
    nk_total = d["ddc_outputs"] / max(1, C)
    direct_flops = C * nk_total * (4.0 * T + 6.0 * D)   # the direct form's count
    mac_ms = d["gpu_ms_ddc_mac"]
    fast = d["ddc_fast_launches"] == launches and launches > 0
    if fast and mac_ms > 0:
        achieved_tf = d["ddc_mac_flop"] / (mac_ms / 1e3) / 1e12
        mac_gbs = d["ddc_mac_bytes"] / (mac_ms / 1e3) / 1e9
    else:
        achieved_tf = direct_flops / (ddc_ms / 1e3) / 1e12 if ddc_ms > 0 else 0.0
        mac_gbs = None
    # the timed fc_mac launches (one per timed block: the first fast group's)
    mac_flop_launch = d["ddc_mac_flop"] / tsteps if fast else None
    mac_bytes_launch = d["ddc_mac_bytes"] / tsteps if fast else None
    mac_ai = (d["ddc_mac_flop"] / d["ddc_mac_bytes"]) if fast and d["ddc_mac_bytes"] > 0 else None
    mac_bound = ("hbm" if mac_ai is not None and mac_ai < RIDGE else "mfma") if fast else "valu"
    if mac_gbs is None:
        mac_gbs = 0.0
    wf_ms = d["gpu_ms_waterfall"]
    post_ms = d["gpu_ms_post"]
    wf_launches = d["waterfall_launches"]
    wf_tlaunches = d["waterfall_timed_launches"]
    # waterfall roofline (HBM-bound, 8 B of cf32 per input sample read once):
    # algorithmic bytes of the frames the timed FFT launches advanced over / their HIP-event time
    wf_fft_ms = d["gpu_ms_waterfall_fft"]
    wf_bytes = 8.0 * d["waterfall_timed_samples"]
    wf_gbs = wf_bytes / (wf_fft_ms / 1e3) / 1e9 if wf_fft_ms > 0 else None
    wf_sub = "wf_fft_l32" if os.environ.get("OWRX_WF_SUB") == "l32" else "wf_fft_q16"
    wf_kernels = (["wf_dif_split", wf_sub, "wf_finalize"] if n_fft > 16384 else
                  ["wf_fft_q16", "wf_finalize"])
    wf_traffic, wf_traffic_src = 0, []
    for kname in wf_kernels:
        b, src = pmc_traffic(kname, args.config)
        wf_traffic = None if (b is None or wf_traffic is None) else wf_traffic + b
        wf_traffic_src.append(src)
    wf_traffic_src = "; ".join(sorted(set(wf_traffic_src)))

    # fc_mac_lds (LDS-DMA ring) where the GEMM grid takes more than one workgroup per CU, fc_mac
    # (register operands) otherwise or with OWRX_FC_MAC=reg: the engine reports which form its
    # timed launches took (and the K slices of the ring form); the PMC traffic is that kernel's
    mac_lds = d["ddc_mac_lds_launches"] > 0
    mac_name = ("fc_mac_lds" if mac_lds else "fc_mac") if fast else "ddc_lds"
    mac_kslices = int(s1["ddc_mac_kslices_max"]) if mac_lds else None
    traffic, traffic_src = pmc_traffic(mac_name + "<", args.config)
    if not fast:
        traffic_src = "direct-form DDC: " + traffic_src
    rt = None
    if rank == 0 and world == 1 and args.realtime_seconds > 0:
        host = stream[hist:hist + min(span, int(fs * 2))].cpu().numpy()
        _log("real-time check")
        rt = realtime_check(Engine, params, fs, n_fft, hop, avg, plist, host,
                            args.realtime_seconds, 1 << 20, args.ddc, wf_batch=wf_batch,
                            wf_cap_ms=args.wf_latency_ms)
    churn = None
    if rank == 0 and world == 1 and args.realtime_seconds > 0 and args.churn_chains > 0:
        host = stream[hist:hist + min(span, int(fs * 2))].cpu().numpy()
        Cc = args.churn_chains
        _log("paced churn check: %d chains" % Cc)
        pc = [params.chain_params(fs, o, cfg["modes"][c % len(cfg["modes"])])
              for c, o in enumerate(carrier_offsets(fs, Cc))]
        churn = realtime_check(Engine, params, fs, n_fft, hop, avg, pc, host,
                               args.realtime_seconds, 1 << 20, args.ddc, churn=True,
                               wf_batch=wf_batch, wf_cap_ms=args.wf_latency_ms)
    cap = None
    if args.capacity_ladder:
        # every rank: 2 s of the same stream on the host (rank 0 slices its own; the others
        # generate it, the synthetic source being deterministic)
        if stream is not None:
            host = stream[hist:hist + min(span, int(fs * 2))].cpu().numpy()
        else:
            host = gen_stream_torch(torch, dev, fs, hist + int(fs * 2), modes, offs)[hist:].cpu().numpy()
        ladder = [int(v) for v in args.capacity_ladder.split(",") if v]

        def agree(v, op):
            if not dist:
                return v
            t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.MIN)
            return float(t.item())
        if dist:
            dist.barrier()
        cap = max_realtime_chains(Engine, params, fs, n_fft, hop, avg, cfg["modes"],
                                  lambda c: carrier_offsets(fs, c), host,
                                  args.capacity_seconds, 1 << 20, ladder, args.ddc, 150.0,
                                  agree=agree, world=world, hold_s=args.capacity_hold_seconds,
                                  wf_batch=wf_batch if world == 1 else 0,
                                  wf_cap_ms=args.wf_latency_ms)
    dropin = None
    if rank == 0 and world == 1 and args.dropin_clients > 0:
        dropin = dropin_check(fs, args.dropin_clients,
                              [int(v) for v in args.dropin_ladder.split(",") if v],
                              args.dropin_seconds, 60.0, 900)
        if args.dropin_c4_clients > 0:
            dropin["c4"] = dropin_c4(args.dropin_c4_clients, args.dropin_seconds, 900)
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            _log("cpu baseline")
            cpu = cpu_baseline(fs, n_fft, hop, avg, plist)
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Msps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "priming_blocks": prime * bps,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": (cfg["label"] % C) + " (waterfall avg %d, hop %d, ADPCM rows; chains "
                            "D=%d, %d taps, frac %.6f, bandpass, squelch, AGC, ADPCM audio)"
                            % (avg, hop, D, T, frac),
                "samp_rate": fs, "fft_size": n_fft, "chains_per_gpu": C,
                "block_samples": block,
                "blocks_per_step": bps,
                "step_samples": bps * block,
                "parallelism": "1 GPU" if world == 1 else
                "IQ broadcast over RCCL from rank 0, %d chains per rank" % C,
                # the same engine set-up at every N (rank 0 holds the waterfall)
                "input_retention_blocks": retention,
                "pipeline_depth_blocks": depth,
                "waterfall_batch_frames_rank0": wf_batch,
                "block_pairing_rank0": bool(pairing),
                "block_pairing_all_ranks": bool(pairing),
                "block_group": group if pairing else 1,
            },
            "value_definition": ("Msamples/s of the ONE wideband IQ stream ingested, at any N: "
                                 "each GPU runs the whole stream (broadcast from rank 0; waterfall "
                                 "on GPU 0) for its own %d chains, so the chain work scales with N "
                                 "(chains_total, chain_msamples_per_s) while the ingested rate "
                                 "does not" % C),
            "iq_msps_stream": round(samples / dt / 1e6, 2),
            "chain_msamples_per_s": round(C * world * samples / dt / 1e6, 1),
            "realtime_factor": round(samples / dt / fs, 1),
            "chains_total": C * world,
            "roofline": {
                "bound": mac_bound,
                "kernel": ("fc_mac (%s): the fast-convolution DDC's per-bin complex GEMM (frames x "
                           "chains x branches) on v_mfma_f32_16x16x4_f32" % mac_name if fast else
                           "ddc_lds (direct polyphase Shift + FirDecimate)"),
                "achieved": round(mac_gbs, 1) if mac_bound == "hbm" else round(achieved_tf, 3),
                "peak": HBM_PEAK_GBS if mac_bound == "hbm" else FP32_PEAK_TFLOPS,
                "unit": "GB/s" if mac_bound == "hbm" else "TFLOP/s",
                "frac": round(mac_gbs / HBM_PEAK_GBS if mac_bound == "hbm"
                              else achieved_tf / FP32_PEAK_TFLOPS, 4),
                "traffic": traffic,
                "mac_form": mac_name,
                "frame_length_M": int(s1.get("ddc_frame_length", 0)) if fast else None,
                "k_slices": mac_kslices,
                "algorithmic_bytes_per_launch": round(mac_bytes_launch) if mac_bytes_launch else None,
                "algorithmic_flop_per_launch": round(mac_flop_launch) if mac_flop_launch else None,
                # per input sample of the stream: W is read once per launch, so pairing halves it
                "algorithmic_bytes_per_input_sample": (round(mac_bytes_launch / (per_engine * block), 2)
                                                       if mac_bytes_launch else None),
                "blocks_per_launch": round(per_engine, 3),
                "arithmetic_intensity_flop_per_byte": round(mac_ai, 2) if mac_ai else None,
                "ridge_flop_per_byte": round(RIDGE, 2),
                "achieved_tflops": round(achieved_tf, 3),
                "mfma_frac": round(achieved_tf / FP32_PEAK_TFLOPS, 4),
                "achieved_hbm_GBps": round(mac_gbs, 1) if mac_gbs else None,
                "hbm_frac": round(mac_gbs / HBM_PEAK_GBS, 4) if mac_gbs else None,
                "note": "bound by the roofline model: the launch's algorithmic flop (8 per complex "
                        "MAC over the frames that carry outputs: 8 M Dp C F) over its algorithmic "
                        "bytes (filter spectra W, unique per chain and bin, + branch spectra U + "
                        "products Y, each moved once) against the ridge 157.3 TFLOP/s / 8 TB/s; "
                        "W's bytes do not depend on the frames per launch, so a 2^20-sample block "
                        "(F ~ 13) sits under the ridge (HBM), a pair of them (block pairing, F ~ 26) "
                        "closer to it and 2^22 (F ~ 31) over it (MFMA).  "
                        "achieved = that bound's quantity / the average launch time from HIP "
                        "events around the kernel on the engine stream; the other figure beside "
                        "it.  traffic = HBM bytes per launch from separate rocprofv3 --pmc "
                        "FETCH_SIZE (x2, gfx950) and WRITE_SIZE passes of this config: "
                        + traffic_src,
                "waterfall": None if wf_gbs is None else {
                    "bound": "hbm",
                    "kernel": " + ".join(wf_kernels) + " (FftChain: Hamming FFT, |X|^2 summed "
                              "over avg frames, 10 log10, FftSwap, quantise)",
                    "achieved": round(wf_gbs, 1),
                    "peak": HBM_PEAK_GBS,
                    "unit": "GB/s",
                    "frac": round(wf_gbs / HBM_PEAK_GBS, 4),
                    "traffic": wf_traffic,
                    # per TIMED launch (the launches the HIP events covered): the bytes are
                    # frames x hop x 8 of exactly those launches, as `achieved` uses
                    "algorithmic_bytes_per_launch": round(wf_bytes / max(1, wf_tlaunches)),
                    "frames_per_launch": round(d["waterfall_timed_samples"] / hop / max(1, wf_tlaunches), 1),
                    "launches": wf_tlaunches,
                    "ms_per_launch": round(wf_fft_ms / max(1, wf_tlaunches), 4),
                    "all_launches": wf_launches,
                    "all_frames_per_launch": round(d["waterfall_frames"] / max(1, wf_launches), 1),
                    "note": "achieved = 8 B x the stream samples the timed launches' frames advanced "
                            "over (frames x hop) / the HIP-event time of those launches (FFT + "
                            "finalize) on stream A; traffic from rocprofv3 PMC passes: "
                            + wf_traffic_src,
                },
            },
            "waterfall_batch": {
                "min_frames": wf_batch,
                "engine_history_samples": hist,
                "latency_cap_s": round(args.wf_latency_ms / 1e3, 3) if wf_batch > 1 else None,
                "row_latency_s": round(s1["wf_row_latency_ms_max"] / 1e3, 4),
                "row_latency_mean_s": round((s1["wf_row_latency_ms_sum"] - s0["wf_row_latency_ms_sum"])
                                            / max(1, d["wf_rows_latency_n"]) / 1e3, 4),
                "batch_stream_span_s": round(wf_batch * hop / fs, 3) if wf_batch > 1 else 0.0,
                "realtime_row_latency_s": round(rt["waterfall_rows"]["latency_ms_max"] / 1e3, 4)
                if rt else None,
                "note": "owrx_waterfall_set_batch: the FFT launches once min_frames frames are "
                        "ready, or when waiting for the next block would hold a ready frame "
                        "longer than latency_cap_s of wall clock (owrx_waterfall_set_latency); "
                        "row_latency_s = the most wall-clock time any row took from the call of "
                        "the block that completed it to the row in the host ring (engine stats, "
                        "the whole run).  Fed faster than real time the batch fills in far less "
                        "than the cap (batch_stream_span_s of stream per launch); at the stream's "
                        "rate (the paced check, realtime_row_latency_s) the cap launches every "
                        "block.  Rows are bit-identical for any batching",
            },
            "ddc": {
                "form": "fast convolution" if fast else "direct",
                "gpu_ms_per_block": round(ddc_ms / tsteps, 4),
                "direct_form_equivalent_TFLOPs": round(direct_flops / (ddc_ms / 1e3) / 1e12, 2)
                if ddc_ms > 0 else None,
                "note": "the whole DDC (branch DFTs + GEMM + inverse DFTs and rotators) against the "
                        "flop count of the direct form it replaces (C outputs (4T + 6D), SURVEY "
                        "8d): what the same outputs would need at that rate",
            },
            # per 2^20-sample block: a timed engine block of a paired engine holds two of them
            "kernels_ms_per_block": {
                "ddc": round(ddc_ms / tblocks, 3),
                "ddc_mac": round(mac_ms / tblocks, 3),
                "waterfall_incl_descriptors": round(wf_ms / tblocks, 3),
                "post_stream_a": round(post_ms / tblocks, 3),
                "post_to_encoder_end": round(d["gpu_ms_serial"] / tsteps, 3),
                "timed_blocks": d["timed_blocks"],
                "blocks_per_engine_block": round(per_engine, 3),
                "blocks_per_engine_block_min_over_ranks": round(per_engine_min, 3),
            },
            "pool_allocs_timed": int(d["pool_allocs"]),
            "host_ms_per_block": {k[8:]: round(d[k] / (args.steps * bps), 3) for k in
                                 ("host_ms_process", "host_ms_wait_input", "host_ms_wait_slots",
                                  "host_ms_wait_rows", "host_ms_build", "host_ms_launch",
                                  "host_ms_collect")},
            "host_ms_per_step_python": {
                "process_device": round(1e3 * host_s["process_t"] / args.steps, 3),
                "step_total": round(1e3 * host_s["drain_t"] / args.steps, 3),
                "blocks_per_step": bps},
            "block_2p22": xblock,
            "realtime": rt,
            "realtime_churn": churn,
            "max_realtime_chains": cap["max_realtime_chains"] if cap else None,
            "max_realtime_chains_60s": cap["max_realtime_chains_held"] if cap else None,
            "capacity": cap,
            "dropin": dropin,
            "cpu_baseline": cpu,
            "output_bytes": out_bytes,
        }
        print(json.dumps(res))
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
