"""Distributed tqdm: progress bars created in tasks/actors are drawn by the driver.

Reference parity: python/ray/experimental/tqdm_ray.py:54 (``tqdm`` with a subset of
tqdm's arguments; bars rendered centrally so concurrent workers do not overwrite each
other). Transport here: a worker-side bar sends its state (rate-limited to one message
per ``flush_interval_s``, always on ``close``) as a fire-and-forget call to one named
collector actor; a driver thread drains the collector and draws every bar with real
``tqdm.tqdm`` at driver-assigned positions. A bar created in the driver draws directly.
"""

from __future__ import annotations

import os
import threading
import time
import uuid
from typing import Iterable, Optional

_COLLECTOR = "_ray_amd_tqdm_collector"
_NAMESPACE = "_ray_amd_internal"


def _in_worker() -> bool:
    from ray_amd._private import worker as _w

    return _w.global_worker.connected and _w.global_worker.mode == _w.WORKER_MODE


class _Collector:
    def __init__(self):
        self._states = {}
        self._dirty = set()

    def update(self, state: dict):
        self._states[state["uuid"]] = state
        self._dirty.add(state["uuid"])

    def drain(self):
        out = [self._states[u] for u in self._dirty]
        self._dirty.clear()
        for s in out:
            if s["closed"]:
                self._states.pop(s["uuid"], None)
        return out


_collector_handle = None
_collector_lock = threading.Lock()


def _collector(create: bool):
    global _collector_handle
    import ray_amd as ray

    with _collector_lock:
        if _collector_handle is not None:
            return _collector_handle
        try:
            h = ray.get_actor(_COLLECTOR, namespace=_NAMESPACE)
        except Exception:
            if not create:
                return None
            h = ray.remote(num_cpus=0)(_Collector).options(
                name=_COLLECTOR, namespace=_NAMESPACE, get_if_exists=True,
                lifetime="detached").remote()
        _collector_handle = h
        return h


class _BarManager:
    """Driver side: one real tqdm per remote bar, positions allocated in creation order."""

    def __init__(self):
        self._bars = {}
        self._lock = threading.Lock()

    def _next_pos(self):
        used = {b.pos for b in self._bars.values()}
        p = 0
        while p in used:
            p += 1
        return p

    def process(self, st: dict):
        import tqdm as real

        with self._lock:
            b = self._bars.get(st["uuid"])
            if b is None:
                if st["closed"] and st["x"] == 0:
                    return
                pos = self._next_pos()
                bar = real.tqdm(total=st["total"], desc=f"{st['desc']} (pid={st['pid']})",
                                position=pos, leave=True)
                bar.pos = pos
                self._bars[st["uuid"]] = b = bar
            b.set_description(f"{st['desc']} (pid={st['pid']})", refresh=False)
            if st["total"] is not None and b.total != st["total"]:
                b.total = st["total"]
            b.update(st["x"] - b.n)
            if st["closed"]:
                b.close()
                self._bars.pop(st["uuid"], None)


_manager = _BarManager()
_poller = None


def _poll_loop(interval: float):
    import ray_amd as ray

    while True:
        time.sleep(interval)
        try:
            if not ray.is_initialized():
                continue
            h = _collector(create=False)
            if h is None:
                continue
            for st in ray.get(h.drain.remote(), timeout=10):
                _manager.process(st)
        except Exception:
            global _collector_handle
            _collector_handle = None  # cluster restarted: look the collector up again


def _ensure_poller(interval: float = 0.25):
    global _poller
    if _poller is None or not _poller.is_alive():
        _poller = threading.Thread(target=_poll_loop, args=(interval,), daemon=True,
                                   name="ray_amd-tqdm")
        _poller.start()


def flush_driver_bars():
    """Draw every pending remote update now (the driver thread does this periodically)."""
    import ray_amd as ray

    h = _collector(create=False)
    if h is not None:
        for st in ray.get(h.drain.remote()):
            _manager.process(st)


class tqdm:
    """tqdm.tqdm subset usable inside ray_amd tasks and actors."""

    DEFAULT_FLUSH_INTERVAL_SECONDS = 1.0

    def __init__(self, iterable: Optional[Iterable] = None, desc: Optional[str] = None,
                 total: Optional[int] = None, position: Optional[int] = None,
                 flush_interval_s: Optional[float] = None):
        if total is None and iterable is not None:
            try:
                total = len(iterable)
            except (TypeError, AttributeError):
                total = None
        self._iterable = iterable
        self._desc = desc or ""
        self._total = total
        self._pos = position or 0
        self._uuid = uuid.uuid4().hex
        self._x = 0
        self._closed = False
        self._flush = (flush_interval_s if flush_interval_s is not None
                       else self.DEFAULT_FLUSH_INTERVAL_SECONDS)
        self._last = 0.0
        self._remote = _in_worker()
        if self._remote:
            self._coll = _collector(create=True)
        else:
            _ensure_poller()
        self._dump(force=True)

    def _state(self) -> dict:
        return {"uuid": self._uuid, "desc": self._desc, "x": self._x, "total": self._total,
                "pos": self._pos, "closed": self._closed, "pid": os.getpid()}

    def _dump(self, force: bool = False):
        now = time.monotonic()
        if not force and now - self._last < self._flush:
            return
        self._last = now
        if self._remote:
            self._coll.update.remote(self._state())
        else:
            _manager.process(self._state())

    def set_description(self, desc):
        self._desc = desc
        self._dump()

    def update(self, n: int = 1):
        self._x += n
        self._dump()

    def refresh(self):
        self._dump(force=True)

    @property
    def total(self) -> Optional[int]:
        return self._total

    @total.setter
    def total(self, total: int):
        self._total = total

    @property
    def n(self) -> int:
        return self._x

    def close(self):
        if self._closed:
            return
        self._closed = True
        try:
            self._dump(force=True)
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __iter__(self):
        if self._iterable is None:
            raise ValueError("No iterable provided")
        for x in iter(self._iterable):
            self.update(1)
            yield x
        self.close()


def safe_print(*args, **kwargs):
    """print() that does not tear the driver's progress bars."""
    import tqdm as real

    real.tqdm.write(" ".join(str(a) for a in args), **kwargs)
