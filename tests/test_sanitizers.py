"""ASan + UBSan run of the host code (CPU only).

oracle/san/Makefile builds oracle/csdr_oracle.c and openwebrx_amd/csrc/design.cpp (the
engine's host-side filter/window/AGC design) with -fsanitize=address,undefined on the host
side only, linked into oracle/san/san_check.cpp, which drives every oracle entry point over
empty, ragged and large inputs and cross-checks design.cpp's taps against the oracle's.
Any sanitizer report aborts the run (-fno-sanitize-recover=all).  GPU code is never
sanitized (not available on the MI355X pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "oracle", "san")
HIPCC = "/opt/rocm/bin/hipcc"
CLANG = "/opt/rocm/llvm/bin/clang"


@pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(CLANG)),
                    reason="ROCm clang/hipcc not present")
def test_oracle_and_design_under_asan_ubsan():
    if shutil.which("make") is None:
        pytest.skip("make not present")
    b = subprocess.run(["make", "-s", "-C", SAN], capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stdout + b.stderr
    env = dict(os.environ)
    # leak checking needs ptrace, which some sandboxes deny; bounds/UB checks stay on
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([os.path.join(ROOT, "oracle", "_san", "san_check")], capture_output=True,
                       text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-4000:]
    assert "san_check ok" in r.stdout
