"""The C-ABI library loads and exports every symbol include/owrx_amd.h declares (no GPU
needed); the binding's prototype table covers the header exactly."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "owrx_amd.h")) as f:
        src = f.read()
    return set(re.findall(r"\b(owrx_[a-z0-9_]+)\s*\(", src))


def test_library_exports_all_header_symbols():
    lib = ctypes.CDLL(os.path.join(ROOT, "openwebrx_amd", "libowrx_amd.so"))
    syms = header_symbols()
    assert len(syms) >= 30
    missing = [s for s in sorted(syms) if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_header():
    from openwebrx_amd import _lib
    assert set(_lib.PROTOTYPES) == header_symbols()


def test_version_and_no_device_is_an_error_not_a_fallback():
    from openwebrx_amd import _lib
    assert _lib.lib.owrx_version().decode().startswith("0.18")
    n = _lib.lib.owrx_device_count()
    assert n > 0 or n == _lib.OWRX_ENODEV


def test_engine_create_without_device_raises():
    import pytest
    from openwebrx_amd import Engine, _lib
    if _lib.lib.owrx_device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(OSError):
        Engine(10e6)


@pytest.mark.parametrize("ctype,cname", [("ChainParams", "owrx_chain_params"),
                                         ("Stats", "owrx_stats")])
def test_struct_layout_matches_header(ctype, cname):
    from openwebrx_amd import _lib
    # int/float fields are 4 bytes, frac_rate is an 8-byte double at offset 16
    assert _lib.ChainParams.frac_rate.offset == 16
    # every field's offset and the size agree with the C compiler's layout of the header
    import shutil
    import subprocess
    import tempfile
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    st = getattr(_lib, ctype)
    names = [n for n, _ in st._fields_]
    prog = ('#include <stdio.h>\n#include <stddef.h>\n#include "owrx_amd.h"\nint main(void){'
            + "".join('printf("%%zu\\n", offsetof(%s, %s));' % (cname, n) for n in names)
            + 'printf("%%zu\\n", sizeof(%s)); return 0;}' % cname)
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        with open(src, "w") as f:
            f.write(prog)
        subprocess.run(["gcc", "-I", inc, src, "-o", exe], check=True)
        got = [int(v) for v in subprocess.run([exe], capture_output=True, text=True,
                                              check=True).stdout.split()]
    want = [getattr(st, n).offset for n in names] + [ctypes.sizeof(st)]
    assert got == want


def test_w_layout_selftest_every_capacity():
    """The fast-convolution DDC's tiled filter spectra (kernels_fcddc.hip fc_w_chain /
    fc_w_branch): for C4's design (D = 5120 -> Dp = 5184) and C3's (D = 833 -> Dp = 864), every
    member slot's entries lie inside its bin's row and no two overlap, at every capacity the
    engine allocates (multiples of the tile up to 4096 members); geometries it never allocates
    are rejected.  Host code: no GPU needed."""
    from openwebrx_amd import _lib
    L = _lib.lib
    for dp in (864, 5184):
        for cap in list(range(32, 1025, 32)) + [2048, 4096]:
            assert L.owrx_selftest_w_layout(dp, cap) == 0, (dp, cap, _lib.last_error())
    assert L.owrx_selftest_w_layout(5184, 130) == _lib.OWRX_EINVAL
    assert L.owrx_selftest_w_layout(5180, 128) == _lib.OWRX_EINVAL
