"""Application metrics: Counter / Gauge / Histogram with tags, exported in Prometheus
text format.

Parity with ``python/ray/util/metrics.py`` (Metric:19, Counter:137, Histogram:187,
Gauge:262: ``set_default_tags``, tag validation, ``info``, picklable metric objects).

Design: the reference records into the C++ OpenCensus/OpenTelemetry pipeline of each
worker and ships to the per-node metrics agent. Here every process keeps its series in
a local registry; a daemon thread pushes a snapshot (only when something changed) to the
raylet over the process's existing raylet connection every ``RAY_AMD_METRICS_INTERVAL_S``
(default 1 s). The raylet merges the snapshots per (process, series) and adds node/system
series (task counts by state, object-store bytes, worker counts); ``prometheus_text()``
and the dashboard's ``/metrics`` endpoint render the merged view.
"""

from __future__ import annotations

import os
import threading
import time
from typing import Dict, Optional, Tuple, Union

_lock = threading.Lock()
_registry: Dict[str, "Metric"] = {}
_dirty = False
_flusher: Optional[threading.Thread] = None

_DEFAULT_BOUNDARIES = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0)


class Metric:
    _kind = "untyped"

    def __init__(self, name: str, description: str = "", tag_keys: Optional[Tuple[str, ...]] = None):
        if len(name) == 0:
            raise ValueError("Empty name is not allowed. Please provide a metric name.")
        self._name = name
        self._description = description
        self._default_tags: Dict[str, str] = {}
        self._tag_keys = tag_keys or tuple()
        if not isinstance(self._tag_keys, tuple):
            raise TypeError(f"tag_keys should be a tuple type, got: {type(self._tag_keys)}")
        for k in self._tag_keys:
            if not isinstance(k, str):
                raise TypeError(f"Tag keys must be str, got {type(k)}.")
        # same (kind, name) in one process = the same series (as the reference's views)
        with _lock:
            prev = _registry.get(f"{self._kind}:{name}")
            if prev is not None:
                self._series = prev._series
            else:
                self._series: Dict[tuple, object] = {}
                _registry[f"{self._kind}:{name}"] = self
        _ensure_flusher()

    def set_default_tags(self, default_tags: Dict[str, str]):
        for k, v in default_tags.items():
            if k not in self._tag_keys:
                raise ValueError(f"Unrecognized tag key {k}.")
            if not isinstance(v, str):
                raise TypeError(f"Tag values must be str, got {type(v)}.")
        self._default_tags = dict(default_tags)
        return self

    def _final_tags(self, tags: Optional[Dict[str, str]]) -> tuple:
        final = dict(self._default_tags)
        final.update(tags or {})
        for k, v in final.items():
            if k not in self._tag_keys:
                raise ValueError(f"Unrecognized tag key {k}.")
            if not isinstance(v, str):
                raise TypeError(f"Tag values must be str, got {type(v)}.")
        missing = set(self._tag_keys) - set(final)
        if missing:
            raise ValueError(f"Missing value for tag key(s): {','.join(sorted(missing))}.")
        return tuple(sorted(final.items()))

    @property
    def info(self):
        return {"name": self._name, "description": self._description,
                "tag_keys": self._tag_keys, "default_tags": self._default_tags}

    def _snapshot(self):
        return {"kind": self._kind, "name": self._name, "description": self._description,
                "series": {k: (list(v) if isinstance(v, list) else v)
                           for k, v in self._series.items()}, **self._extra()}

    def _extra(self):
        return {}

    def __reduce__(self):
        return (type(self)._rebuild, (self._name, self._description, self._tag_keys,
                                      self._default_tags, self._extra()))

    @classmethod
    def _rebuild(cls, name, description, tag_keys, default_tags, extra):
        m = cls(name, description, tag_keys=tag_keys, **extra)
        m._default_tags = default_tags
        return m


def _mark():
    global _dirty
    _dirty = True


class Counter(Metric):
    """Monotonically increasing cumulative count."""

    _kind = "counter"

    def inc(self, value: Union[int, float] = 1.0, tags: Dict[str, str] = None):
        if value <= 0:
            raise ValueError(f"value must be >0, got {value}")
        key = self._final_tags(tags)
        with _lock:
            self._series[key] = self._series.get(key, 0.0) + float(value)
        _mark()


class Gauge(Metric):
    """Last value wins."""

    _kind = "gauge"

    def set(self, value: Union[int, float], tags: Dict[str, str] = None):
        if value is None:
            return
        key = self._final_tags(tags)
        with _lock:
            self._series[key] = float(value)
        _mark()


class Histogram(Metric):
    """Bucketed distribution (cumulative buckets + sum + count, Prometheus style)."""

    _kind = "histogram"

    def __init__(self, name: str, description: str = "", boundaries=None, tag_keys=None):
        boundaries = list(boundaries or _DEFAULT_BOUNDARIES)
        if not boundaries:
            raise ValueError("boundaries must be non-empty")
        for b in boundaries:
            if b <= 0:
                raise ValueError("Invalid `boundaries` argument: boundaries must be > 0")
        if sorted(boundaries) != boundaries:
            raise ValueError("boundaries must be sorted ascending")
        self.boundaries = boundaries
        super().__init__(name, description, tag_keys)

    def observe(self, value: Union[int, float], tags: Dict[str, str] = None):
        key = self._final_tags(tags)
        with _lock:
            s = self._series.get(key)
            if s is None:
                s = self._series[key] = [0] * (len(self.boundaries) + 1) + [0.0, 0]
            i = 0
            nb = len(self.boundaries)
            while i < nb and value > self.boundaries[i]:
                i += 1
            s[i] += 1
            s[-2] += float(value)
            s[-1] += 1
        _mark()

    def _extra(self):
        return {"boundaries": self.boundaries}

    @property
    def info(self):
        d = super().info
        d["boundaries"] = self.boundaries
        return d


# ---------------------------------------------------------------------------- export
def _snapshot_all():
    with _lock:
        return [m._snapshot() for m in _registry.values()]


def flush_now():
    """Push this process's metrics to the raylet immediately (tests / shutdown)."""
    global _dirty
    from ray_amd._private import worker as _w

    cw = _w.global_worker.core
    if cw is None:
        return False
    _dirty = False
    cw.notify_raylet("metrics", os.getpid(), _snapshot_all())
    return True


def _flush_loop():
    interval = float(os.environ.get("RAY_AMD_METRICS_INTERVAL_S", "1.0"))
    while True:
        time.sleep(interval)
        if _dirty:
            try:
                flush_now()
            except Exception:
                pass


def _ensure_flusher():
    global _flusher
    if _flusher is None:
        with _lock:
            if _flusher is None:
                _flusher = threading.Thread(target=_flush_loop, daemon=True,
                                            name="ray_amd-metrics")
                _flusher.start()


def _esc(v: str) -> str:
    return v.replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def _labels(pairs) -> str:
    if not pairs:
        return ""
    return "{" + ",".join(f'{k}="{_esc(str(v))}"' for k, v in pairs) + "}"


def render_prometheus(snapshots) -> str:
    """Prometheus text exposition of merged metric snapshots.

    ``snapshots``: list of metric dicts (as produced by ``_snapshot``) possibly from many
    processes; same-named counters/histograms are summed, gauges take the last value."""
    merged: Dict[str, dict] = {}
    for m in snapshots:
        name = "ray_" + m["name"] if not m["name"].startswith("ray_") else m["name"]
        e = merged.setdefault(name, {"kind": m["kind"], "description": m["description"],
                                     "boundaries": m.get("boundaries"), "series": {}})
        for key, v in m["series"].items():
            key = tuple(tuple(p) for p in key)
            if m["kind"] == "histogram":
                cur = e["series"].get(key)
                e["series"][key] = list(v) if cur is None else [a + b for a, b in zip(cur, v)]
            elif m["kind"] == "counter":
                e["series"][key] = e["series"].get(key, 0.0) + v
            else:
                e["series"][key] = v
    out = []
    for name in sorted(merged):
        e = merged[name]
        kind = e["kind"] if e["kind"] != "untyped" else "gauge"
        out.append(f"# HELP {name} {e['description'] or name}")
        out.append(f"# TYPE {name} {kind}")
        for key, v in sorted(e["series"].items()):
            if kind == "histogram":
                cum = 0
                for b, c in zip(e["boundaries"], v):
                    cum += c
                    out.append(f"{name}_bucket{_labels(key + (('le', repr(float(b))),))} {cum}")
                cum += v[len(e["boundaries"])]
                out.append(f"{name}_bucket{_labels(key + (('le', '+Inf'),))} {cum}")
                out.append(f"{name}_sum{_labels(key)} {v[-2]}")
                out.append(f"{name}_count{_labels(key)} {v[-1]}")
            else:
                out.append(f"{name}{_labels(key)} {v}")
    return "\n".join(out) + "\n"


def prometheus_text() -> str:
    """Cluster-wide metrics (all processes + node/system series) in Prometheus format."""
    from ray_amd._private import worker as _w

    cw = _w._check_connected()
    flush_now()
    return render_prometheus(cw.call_raylet("get_metrics"))
