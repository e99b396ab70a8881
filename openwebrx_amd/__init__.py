"""MI355X-native IQ backend for OpenWebRX (waterfall FFT path + client demod chains).

The compute path is libowrx_amd.so (hand-written HIP for gfx950, C ABI in
include/owrx_amd.h); this package is its Python side.  ``pycsdr`` at the repository root is
the drop-in replacement of the reference's pycsdr extension built on top of it.
"""
from . import _lib, params  # noqa: F401  (raises ImportError if the HIP library is missing)
from .engine import Chain, Engine, Module, Waterfall, device_count  # noqa: F401

__version__ = "0.18.99"
