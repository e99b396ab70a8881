import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")


def pytest_collection_modifyitems(config, items):
    # torch bundles its own HIP runtime under the same soname as the engine's (/opt/rocm): the
    # first one loaded serves both, and torch does not initialise on ROCm 7.2's.  GPU tests use
    # torch for device buffers, so it loads before any test loads libowrx_amd.so.
    if any(item.get_closest_marker("gpu") for item in items):
        try:
            import torch  # noqa: F401
        except ImportError:
            pass


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def parity_report():
    """report(test, **metrics): appends one JSON line to gpurun_out/parity_metrics.jsonl (the
    measured parity figures -- exact-match fractions, rel-RMS -- kept beside the pass/fail)."""
    import json
    path = os.path.join(ROOT, "gpurun_out", "parity_metrics.jsonl")

    def report(test, **metrics):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps({"test": test, **metrics}) + "\n")
        print(test, metrics)
    return report
