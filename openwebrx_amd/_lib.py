"""ctypes binding of libowrx_amd.so (include/owrx_amd.h).

The library is the only compute path: there is no CPU fallback.  If the shared object is
missing or cannot be loaded this module raises at import time, and every engine call that
fails on the device raises OSError / ValueError like the pycsdr extension it replaces
(csdr/chain/__init__.py:60-84 relies on ValueError for format mismatches).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OWRX_AMD_LIB", os.path.join(_HERE, "libowrx_amd.so"))

OWRX_OK = 0
OWRX_EIO = -5
OWRX_EAGAIN = -11
OWRX_ENOMEM = -12
OWRX_EINVAL = -22
OWRX_ENOSPC = -28
OWRX_ENODEV = -19
OWRX_ETIMEDOUT = -110  # a GPU wait exceeded the stall timeout (engine failed)

DEMOD_NFM, DEMOD_AM, DEMOD_SSB, DEMOD_WFM, DEMOD_SAM = 0, 1, 2, 3, 4
OUT_S16, OUT_ADPCM, OUT_F32, OUT_IQ, OUT_SEL = 0, 1, 2, 3, 4
AGC_FAST, AGC_SLOW, AGC_MID, AGC_LAGGY = 0, 1, 2, 3

MOD_FMDEMOD = 1
MOD_AMDEMOD = 2
MOD_REALPART = 3
MOD_LIMIT = 4
MOD_DCBLOCK = 5
MOD_DEEMPH = 6
MOD_AGC = 7
MOD_CONVERT_F_S16 = 8
MOD_ADPCM = 9
MOD_FFTSWAP = 10
MOD_FFTADPCM = 11
MOD_CONVERT_CS16_CF32 = 12
MOD_GAIN = 13
MOD_SHIFT = 14
MOD_BANDPASS = 15
MOD_AUDIO_RESAMPLER = 16
MOD_AFC = 17


class ChainParams(ctypes.Structure):
    _fields_ = [
        ("shift_rate", ctypes.c_float),
        ("decimation", ctypes.c_int32),
        ("transition", ctypes.c_float),
        ("cutoff", ctypes.c_float),
        ("frac_rate", ctypes.c_double),
        ("bandpass", ctypes.c_int32),
        ("bp_low", ctypes.c_float),
        ("bp_high", ctypes.c_float),
        ("bp_transition", ctypes.c_float),
        ("sq_length", ctypes.c_int32),
        ("sq_decimation", ctypes.c_int32),
        ("sq_hang", ctypes.c_int32),
        ("sq_flush", ctypes.c_int32),
        ("sq_report", ctypes.c_int32),
        ("sq_level", ctypes.c_float),
        ("demod", ctypes.c_int32),
        ("agc_profile", ctypes.c_int32),
        ("agc_initial_gain", ctypes.c_float),
        ("agc_max_gain", ctypes.c_float),
        ("audio_rate", ctypes.c_int32),
        ("output", ctypes.c_int32),
        ("deemph_tau", ctypes.c_float),
        ("if_rate", ctypes.c_double),
        ("nr_enabled", ctypes.c_int32),
        ("nr_threshold", ctypes.c_float),
        ("afc_update", ctypes.c_int32),
        ("afc_sample", ctypes.c_int32),
        ("audio_gain", ctypes.c_float),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("samples_in", ctypes.c_int64),
        ("blocks", ctypes.c_int64),
        ("ddc_outputs", ctypes.c_int64),
        ("waterfall_rows", ctypes.c_int64),
        ("audio_bytes", ctypes.c_int64),
        ("overruns", ctypes.c_int64),
        ("gpu_ms_ddc", ctypes.c_double),
        ("gpu_ms_waterfall", ctypes.c_double),
        ("gpu_ms_post", ctypes.c_double),
        ("ddc_launches", ctypes.c_int64),
        ("waterfall_launches", ctypes.c_int64),
        ("ddc_fast_launches", ctypes.c_int64),
        ("gpu_ms_ddc_mac", ctypes.c_double),
        ("ddc_mac_flop", ctypes.c_double),
        ("ddc_mac_bytes", ctypes.c_double),
        ("gpu_ms_serial", ctypes.c_double),
        ("host_ms_process", ctypes.c_double),
        ("host_ms_wait_input", ctypes.c_double),
        ("host_ms_wait_slots", ctypes.c_double),
        ("host_ms_wait_rows", ctypes.c_double),
        ("waterfall_frames", ctypes.c_int64),
        ("waterfall_samples", ctypes.c_int64),
        ("gpu_ms_waterfall_fft", ctypes.c_double),
        ("waterfall_timed_samples", ctypes.c_int64),
        ("timed_blocks", ctypes.c_int64),
        ("pipeline_drains", ctypes.c_int64),
        ("host_ms_build", ctypes.c_double),
        ("host_ms_launch", ctypes.c_double),
        ("host_ms_collect", ctypes.c_double),
        ("wf_row_latency_ms_max", ctypes.c_double),
        ("wf_row_latency_ms_sum", ctypes.c_double),
        ("wf_rows_latency_n", ctypes.c_int64),
        ("ddc_mac_lds_launches", ctypes.c_int64),
        ("ddc_mac_kslices_max", ctypes.c_int64),
        ("pool_allocs", ctypes.c_int64),
        ("gpu_ms_waterfall_fft_max", ctypes.c_double),
        ("waterfall_timed_launches", ctypes.c_int64),
        ("host_ms_drain_wait", ctypes.c_double),
        ("host_ms_drain_copy", ctypes.c_double),
        ("ddc_frame_length", ctypes.c_int64),
    ]


_vp = ctypes.c_void_p
_i32 = ctypes.c_int
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_f64 = ctypes.c_double
_pi32 = ctypes.POINTER(ctypes.c_int)
_pi64 = ctypes.POINTER(ctypes.c_int64)

# name: (restype, argtypes)  -- every symbol declared in include/owrx_amd.h
PROTOTYPES = {
    "owrx_version": (ctypes.c_char_p, []),
    "owrx_last_error": (ctypes.c_char_p, []),
    "owrx_device_count": (_i32, []),
    "owrx_engine_create": (_i32, [_i32, _f64, _i64, ctypes.POINTER(_vp)]),
    "owrx_engine_create_ex": (_i32, [_i32, _f64, _i64, _i64, ctypes.POINTER(_vp)]),
    "owrx_engine_destroy": (_i32, [_vp]),
    "owrx_engine_history": (_i64, [_vp]),
    "owrx_engine_max_block": (_i64, [_vp]),
    "owrx_push_iq": (_i32, [_vp, _vp, _i64]),
    "owrx_push_iq_cs16": (_i32, [_vp, _vp, _i64, _f32]),
    "owrx_process_device": (_i32, [_vp, _vp, _i64]),
    "owrx_wait_stream": (_i32, [_vp, _vp]),
    "owrx_ingest_buffer": (_i32, [_vp, ctypes.POINTER(_vp), _pi64]),
    "owrx_commit": (_i32, [_vp, _i64]),
    "owrx_sync": (_i32, [_vp]),
    "owrx_waterfall_create": (_i32, [_vp, _i32, _i32, _i32, _f32, _i32, _pi32]),
    "owrx_waterfall_set": (_i32, [_vp, _i32, _i32, _i32, _i32]),
    "owrx_waterfall_set_batch": (_i32, [_vp, _i32, _i32, _i64]),
    "owrx_waterfall_set_latency": (_i32, [_vp, _i32, _f64]),
    "owrx_set_input_retention": (_i32, [_vp, _i32]),
    "owrx_set_block_pairing": (_i32, [_vp, _i32]),
    "owrx_set_block_group": (_i32, [_vp, _i32]),
    "owrx_set_pipeline_depth": (_i32, [_vp, _i32]),
    "owrx_set_stall_timeout": (_i32, [_vp, _i64]),
    "owrx_debug_stall": (_i32, [_vp, _i32, _i64]),
    "owrx_selftest_w_layout": (_i32, [_i32, _i32]),
    "owrx_waterfall_destroy": (_i32, [_vp, _i32]),
    "owrx_waterfall_row_bytes": (_i64, [_vp, _i32]),
    "owrx_waterfall_round_frames": (_i32, [_vp, _i32]),
    "owrx_waterfall_read": (_i64, [_vp, _i32, _vp, _i64]),
    "owrx_chain_create": (_i32, [_vp, ctypes.POINTER(ChainParams), _pi32]),
    "owrx_chain_destroy": (_i32, [_vp, _i32]),
    "owrx_chain_set_shift_rate": (_i32, [_vp, _i32, _f32]),
    "owrx_chain_set_bandpass": (_i32, [_vp, _i32, _i32, _f32, _f32]),
    "owrx_chain_set_squelch_level": (_i32, [_vp, _i32, _f32]),
    "owrx_chain_set_noise_filter": (_i32, [_vp, _i32, _i32, _f32]),
    "owrx_chain_read_audio": (_i64, [_vp, _i32, _vp, _i64]),
    "owrx_chain_read_smeter": (_i64, [_vp, _i32, _vp, _i64]),
    "owrx_chain_origin": (_i64, [_vp, _i32]),
    "owrx_chain_set_secondary_fft": (_i32, [_vp, _i32, _i32, _i32, _i32, _f32, _i32]),
    "owrx_chain_secondary_fft_row_bytes": (_i64, [_vp, _i32]),
    "owrx_chain_read_secondary_fft": (_i64, [_vp, _i32, _vp, _i64]),
    "owrx_set_debug": (_i32, [_vp, _i32]),
    "owrx_chain_read_debug": (_i64, [_vp, _i32, _i32, _vp, _i64]),
    "owrx_get_stats": (_i32, [_vp, ctypes.POINTER(Stats)]),
    "owrx_set_timing": (_i32, [_vp, _i32]),
    "owrx_set_ddc_mode": (_i32, [_vp, _i32]),
    "owrx_module_set": (_i32, [_vp, _f64, _f64, _f64]),
    "owrx_chain_set_taps": (_i32, [_vp, _i32, _i32, _i32]),
    "owrx_chain_read_tap": (_i64, [_vp, _i32, _i32, _vp, _i64]),
    "owrx_synth_iq": (_i32, [_i32, _vp, _i64, _i64, _f64, _i32, _vp, _vp, ctypes.c_uint64, _f32, _f32]),
    "owrx_chains_read_audio": (_i64, [_vp, _i32, _pi32, _vp, _i64, _pi64]),
    "owrx_chains_read_smeter": (_i64, [_vp, _i32, _pi32, _vp, _i64, _pi64]),
    "owrx_module_create": (_i32, [_i32, _i32, _f64, _f64, _f64, ctypes.POINTER(_vp)]),
    "owrx_module_destroy": (_i32, [_vp]),
    "owrx_module_process": (_i64, [_vp, _vp, _i64, _vp, _i64]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libowrx_amd.so not found at %s: build it with `python -c 'import __graft_entry__ as g; "
            "g.build()'` (hipcc --offload-arch=gfx950).  There is no CPU fallback." % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in PROTOTYPES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    e = lib.owrx_last_error()
    return e.decode() if e else ""


def check(rc, what=""):
    """Map negative return codes to the exceptions the pycsdr callers expect."""
    if rc is None or rc >= 0:
        return rc
    msg = "%s: %s (rc=%d)" % (what, last_error(), rc)
    if rc == OWRX_EINVAL:
        raise ValueError(msg)
    if rc == OWRX_ENOMEM:
        raise MemoryError(msg)
    if rc == OWRX_ETIMEDOUT:
        raise TimeoutError(-rc, msg)  # an OSError subclass: the shim's failure path catches it
    raise OSError(-rc, msg)
