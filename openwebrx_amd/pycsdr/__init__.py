"""Drop-in mirror of the `pycsdr` extension (pycsdr.modules + pycsdr.types)
backed by libowrx_amd.so.  `install()` registers it under the name `pycsdr` so the
reference's csdr/chain/*.py and owrx/*.py import it unchanged."""
import sys

from . import modules, types

__all__ = ["modules", "types", "install"]


def install():
    """Make `import pycsdr`, `pycsdr.modules`, `pycsdr.types` resolve to this package."""
    sys.modules["pycsdr"] = sys.modules[__name__]
    sys.modules["pycsdr.modules"] = modules
    sys.modules["pycsdr.types"] = types
