"""pycsdr.types mirror: the enums the reference imports (csdr/chain/*.py, owrx/dsp.py:15,
owrx/form/input/__init__.py:5,344)."""
from enum import Enum

from .. import _lib


class Format(Enum):
    """Sample formats of csdr buffers (CHAR, SHORT, FLOAT, COMPLEX_FLOAT,
    COMPLEX_SHORT)."""
    CHAR = "char"
    SHORT = "short"
    FLOAT = "float"
    COMPLEX_FLOAT = "complex_float"
    COMPLEX_SHORT = "complex_short"

    @property
    def itemsize(self):
        return _ITEMSIZE[self]


_ITEMSIZE = {Format.CHAR: 1, Format.SHORT: 2, Format.FLOAT: 4, Format.COMPLEX_FLOAT: 8,
             Format.COMPLEX_SHORT: 4}


class AgcProfile(Enum):
    """Agc profiles; constructible from the config string (owrx/dsp.py:619,
    owrx/config/defaults.py:438 "Fast") and iterable for the settings UI
    (owrx/form/input/__init__.py:344).  CHANGELOG.md:107-108 adds MID and LAGGY."""
    FAST = "Fast"
    SLOW = "Slow"
    MID = "Mid"
    LAGGY = "Laggy"

    @property
    def engine_id(self):
        return {AgcProfile.FAST: _lib.AGC_FAST, AgcProfile.SLOW: _lib.AGC_SLOW,
                AgcProfile.MID: _lib.AGC_MID, AgcProfile.LAGGY: _lib.AGC_LAGGY}[self]
