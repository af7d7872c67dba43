"""Distributed tracing of tasks and actor calls (reference: python/ray/util/tracing/
tracing_helper.py, which wraps remote calls in OpenTelemetry spans).

OpenTelemetry is not installed here, so ray_amd records the same span tree itself: with
tracing enabled (``ray_amd.init(_tracing_startup_hook=...)``, e.g. ``setup_local_tmp_tracing``)
every ``.remote()`` call records a CLIENT span ``"<name> ray.remote"`` in the caller and
the execution a SERVER span ``"<name> ray.remote_worker"`` in the worker, whose parent is
the submit span; calls made inside a task nest under its span, across processes and
nodes (the trace context travels in the task spec). ``span(name)`` adds user spans.

Spans are JSON lines in ``<export dir>/<pid>.jsonl`` (OpenTelemetry-like fields: name,
context.trace_id / span_id, parent_id, kind, start_time / end_time in ns, attributes,
status). ``read_spans(dir)`` loads them. Nothing is recorded while tracing is off; a
task spec then carries no trace field and workers do no tracing work."""

from __future__ import annotations

import contextlib
import glob
import json
import os
import secrets
import threading
import time
from typing import Any, Dict, List, Optional

ENABLED = False
_dir: Optional[str] = None
_lock = threading.Lock()
_file = None
_local = threading.local()


def enable(export_dir: str) -> None:
    global ENABLED, _dir, _file
    with _lock:
        os.makedirs(export_dir, exist_ok=True)
        if _dir != export_dir and _file is not None:
            _file.close()
            _file = None
        _dir = export_dir
        ENABLED = True


def disable() -> None:
    global ENABLED, _file
    with _lock:
        ENABLED = False
        if _file is not None:
            _file.close()
            _file = None


def is_enabled() -> bool:
    return ENABLED


def _write(span: dict) -> None:
    global _file
    with _lock:
        if _dir is None:
            return
        if _file is None:
            _file = open(os.path.join(_dir, f"{os.getpid()}.jsonl"), "a", buffering=1)
        _file.write(json.dumps(span) + "\n")


def _stack() -> list:
    s = getattr(_local, "stack", None)
    if s is None:
        s = _local.stack = []
    return s


def _current():
    s = _stack()
    return s[-1] if s else None


def _span(name, kind, trace_id, parent_id, attrs) -> dict:
    return {"name": name, "context": {"trace_id": trace_id, "span_id": secrets.token_hex(8)},
            "parent_id": parent_id, "kind": kind, "start_time": time.time_ns(),
            "end_time": None, "attributes": dict(attrs), "status": {"status_code": "UNSET"}}


def inject(spec: dict, kind: str = "function") -> None:
    """Caller side of ``.remote()``: record the submit span and put the trace context
    into the task spec."""
    cur = _current()
    trace_id = cur["context"]["trace_id"] if cur else secrets.token_hex(16)
    parent = cur["context"]["span_id"] if cur else None
    name = spec.get("name") or spec.get("method") or "task"
    sp = _span(f"{name} ray.remote", "CLIENT", trace_id, parent,
               {"ray.remote": kind, "ray.function": name, "ray.pid": os.getpid(),
                "ray.task_id": spec["tid"].hex() if isinstance(spec.get("tid"), bytes)
                else str(spec.get("tid"))})
    sp["end_time"] = time.time_ns()
    sp["status"]["status_code"] = "OK"
    _write(sp)
    spec["trace"] = {"t": trace_id, "p": sp["context"]["span_id"], "d": _dir}


def on_execute_start(spec: dict, actor_id=None):
    tr = spec.get("trace")
    if not tr:
        return None
    if not ENABLED and tr.get("d"):
        enable(tr["d"])  # the worker joins the caller's trace export
    name = spec.get("name") or spec.get("method") or "task"
    attrs = {"ray.function": name, "ray.pid": os.getpid(),
             "ray.task_id": spec["tid"].hex() if isinstance(spec.get("tid"), bytes)
             else str(spec.get("tid"))}
    if actor_id is not None:
        attrs["ray.actor_id"] = actor_id.hex() if isinstance(actor_id, bytes) else str(actor_id)
    sp = _span(f"{name} ray.remote_worker", "SERVER", tr["t"], tr["p"], attrs)
    _stack().append(sp)
    return sp


def on_execute_end(sp, error: bool = False) -> None:
    if sp is None:
        return
    st = _stack()
    if st and st[-1] is sp:
        st.pop()
    sp["end_time"] = time.time_ns()
    sp["status"]["status_code"] = "ERROR" if error else "OK"
    _write(sp)


@contextlib.contextmanager
def span(name: str, **attributes: Any):
    """A user span, nested under the current task's (or an enclosing user) span."""
    if not ENABLED:
        yield None
        return
    cur = _current()
    sp = _span(name, "INTERNAL", cur["context"]["trace_id"] if cur else secrets.token_hex(16),
               cur["context"]["span_id"] if cur else None, attributes)
    _stack().append(sp)
    err = False
    try:
        yield sp
    except BaseException:
        err = True
        raise
    finally:
        on_execute_end(sp, err)


def read_spans(export_dir: str) -> List[Dict[str, Any]]:
    out = []
    for f in sorted(glob.glob(os.path.join(export_dir, "*.jsonl"))):
        with open(f) as fh:
            out.extend(json.loads(line) for line in fh if line.strip())
    return out
