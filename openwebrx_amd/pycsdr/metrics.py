"""The GPU engines' counters as OpenWebRX metrics (owrx/metrics.py:29-70).

register(metrics) adds DirectMetric entries under "gpu." to the reference's Metrics registry
(owrx.metrics.Metrics.getSharedInstance() by default); the values are summed over every engine
of every source buffer the shim drives, and read when the metrics page asks
(getHierarchicalMetrics / getFlatMetrics).  "gpu.failed" counts drivers in the FAILED state.

A maintainer calls it once at start-up, e.g. next to the pycsdr install:

    from openwebrx_amd.pycsdr import metrics
    metrics.register()
"""
from . import _graph

# engine counter -> metric name
COUNTERS = {
    "samples_in": "gpu.samples_in",
    "blocks": "gpu.blocks",
    "ddc_outputs": "gpu.ddc_outputs",
    "waterfall_rows": "gpu.waterfall_rows",
    "audio_bytes": "gpu.audio_bytes",
    "overruns": "gpu.overruns",
}


def _drivers():
    with _graph._lock:
        return list(_graph._drivers.values())


def totals():
    """Engine counters summed over every driver (dict: metric name -> value)."""
    out = {name: 0 for name in COUNTERS.values()}
    out.update({"gpu.engines": 0, "gpu.segments": 0, "gpu.failed": 0})
    for drv in _drivers():
        out["gpu.failed"] += drv.state == "FAILED"
        out["gpu.segments"] += len(drv.segments)
        for eng in list(drv.engines.values()):
            if eng.handle is None:
                continue
            out["gpu.engines"] += 1
            st = eng.stats()
            for k, name in COUNTERS.items():
                out[name] += int(st[k])
    return out


def register(metrics=None):
    """Add one DirectMetric per counter to `metrics` (default: the shared owrx.metrics
    registry).  Returns the metric names added."""
    if metrics is None:
        from owrx.metrics import Metrics
        metrics = Metrics.getSharedInstance()
    try:
        from owrx.metrics import DirectMetric
    except ImportError:  # a registry outside OpenWebRX: anything with getValue() will do
        class DirectMetric:
            def __init__(self, getter):
                self.getter = getter

            def getValue(self):
                return self.getter()
    names = list(COUNTERS.values()) + ["gpu.engines", "gpu.segments", "gpu.failed"]
    for name in names:
        metrics.addMetric(name, DirectMetric(lambda name=name: totals()[name]))
    return names
