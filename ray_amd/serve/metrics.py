"""Serve application metrics (reference: python/ray/serve/metrics.py): ``util.metrics``
Counter / Gauge / Histogram that, inside a replica, tag every sample with the replica's
``deployment``, ``replica`` and ``application`` (and the request's ``route`` when the
caller passes it), exported through the same Prometheus text endpoint."""

from __future__ import annotations

from typing import Dict, Optional, Tuple

from ray_amd.util import metrics as _m

_DEFAULT_KEYS = ("deployment", "replica", "application", "route")


def _context_tags() -> Dict[str, str]:
    from ray_amd.serve import context

    rc = context._replica_ctx
    if rc is None:
        return {}
    return {"deployment": rc.deployment, "replica": rc.replica_tag,
            "application": rc.app_name}


class _ServeMetric:
    @classmethod
    def _rebuild(cls, name, description, tag_keys, default_tags, extra):
        user_keys = tuple(k for k in tag_keys if k not in _DEFAULT_KEYS)
        m = cls(name, description, tag_keys=user_keys, **extra)
        m._default_tags = default_tags
        return m

    def _init_tags(self, tag_keys):
        keys = tuple(tag_keys or ())
        for k in keys:
            if k in _DEFAULT_KEYS:
                raise ValueError(f"'{k}' is a reserved Serve metric tag key")
        return keys + _DEFAULT_KEYS

    def _tags(self, tags: Optional[Dict[str, str]]) -> Dict[str, str]:
        out = dict(_context_tags())
        out.setdefault("route", "")
        out.update(tags or {})
        return out


class Counter(_ServeMetric, _m.Counter):
    def __init__(self, name: str, description: str = "",
                 tag_keys: Optional[Tuple[str, ...]] = None):
        _m.Counter.__init__(self, name, description, self._init_tags(tag_keys))

    def inc(self, value=1.0, tags: Dict[str, str] = None):
        _m.Counter.inc(self, value, self._tags(tags))


class Gauge(_ServeMetric, _m.Gauge):
    def __init__(self, name: str, description: str = "",
                 tag_keys: Optional[Tuple[str, ...]] = None):
        _m.Gauge.__init__(self, name, description, self._init_tags(tag_keys))

    def set(self, value, tags: Dict[str, str] = None):
        _m.Gauge.set(self, value, self._tags(tags))


class Histogram(_ServeMetric, _m.Histogram):
    def __init__(self, name: str, description: str = "", boundaries=None,
                 tag_keys: Optional[Tuple[str, ...]] = None):
        _m.Histogram.__init__(self, name, description, boundaries, self._init_tags(tag_keys))

    def observe(self, value, tags: Dict[str, str] = None):
        _m.Histogram.observe(self, value, self._tags(tags))
