"""Durable workflows over ``ray_amd.dag``.

Parity with ``python/ray/workflow/api.py`` (init:34, run:123, run_async:177, resume:243,
get_output:320, list_all:381, resume_all:502, get_status:577, wait_for_event:607,
sleep:635, get_metadata:649, cancel:712, delete:745, continuation:776, options:797) and
the WorkflowStatus of ``workflow/common.py:81``.

Execution model: ``run_async`` launches ONE runner task that walks the DAG; every
FunctionNode becomes a step task that (1) returns its checkpoint immediately if the step
already committed one, (2) otherwise runs the user function and atomically commits the
output (write-temp + rename) in the worker before returning. Upstream results flow as
ObjectRefs, so independent steps run in parallel across the cluster. A step that returns
``workflow.continuation(dag)`` expands that sub-DAG in place (dynamic workflows); its
final value becomes the step's checkpoint. Resume = re-run the stored DAG: committed steps
are skipped. Storage is a plain directory tree:

    <storage>/<workflow_id>/workflow.json      status, timestamps, user metadata
    <storage>/<workflow_id>/dag.pkl            the DAG + its inputs (for resume)
    <storage>/<workflow_id>/steps/<task_id>/   output.pkl, meta.json
    <storage>/<workflow_id>/output.pkl         final output
"""

from __future__ import annotations

import asyncio
import json
import os
import tempfile
import time
import uuid
from enum import Enum
from typing import Any, Dict, List, Optional, Tuple

import cloudpickle

import ray_amd as ray
from ray_amd.dag import DAGNode, FunctionNode, InputAttributeNode, InputNode, MultiOutputNode

_META_KEY = "workflow.io/options"
_storage_root: Optional[str] = None


class WorkflowStatus(str, Enum):
    NONE = "NONE"
    RUNNING = "RUNNING"
    CANCELED = "CANCELED"
    SUCCESSFUL = "SUCCESSFUL"
    FAILED = "FAILED"
    RESUMABLE = "RESUMABLE"
    PENDING = "PENDING"

    @classmethod
    def non_terminating_status(cls):
        return cls.RUNNING, cls.PENDING


class WorkflowError(Exception):
    pass


class WorkflowExecutionError(WorkflowError):
    def __init__(self, workflow_id: str):
        super().__init__(f"Workflow[id={workflow_id}] failed during execution.")
        self.workflow_id = workflow_id


class WorkflowCancellationError(WorkflowError):
    def __init__(self, workflow_id: str):
        super().__init__(f"Workflow[id={workflow_id}] is cancelled during execution.")
        self.workflow_id = workflow_id


class WorkflowNotFoundError(WorkflowError):
    def __init__(self, workflow_id: str):
        super().__init__(f"Workflow[id={workflow_id}] was referenced but doesn't exist.")
        self.workflow_id = workflow_id


# ---------------------------------------------------------------------------- storage
def init(storage: Optional[str] = None, *, max_running_workflows=None,
         max_pending_workflows=None) -> None:
    """Set the storage root (reference: workflow.init). Defaults to
    ``$RAY_AMD_WORKFLOW_STORAGE`` or ``/tmp/ray_amd_workflows``."""
    global _storage_root
    if storage and storage.startswith("file://"):
        storage = storage[len("file://"):]
    _storage_root = os.path.abspath(storage or os.environ.get("RAY_AMD_WORKFLOW_STORAGE") or
                                    os.path.join(tempfile.gettempdir(), "ray_amd_workflows"))
    os.makedirs(_storage_root, exist_ok=True)


def _root() -> str:
    if _storage_root is None:
        init()
    return _storage_root


def _wdir(root, wid):
    return os.path.join(root, wid)


def _atomic_write(path: str, data: bytes) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = f"{path}.{uuid.uuid4().hex[:8]}.tmp"
    with open(tmp, "wb") as f:
        f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def _read_json(path, default=None):
    try:
        with open(path) as f:
            return json.load(f)
    except (FileNotFoundError, json.JSONDecodeError):
        return default


def _set_wf(root, wid, **fields):
    p = os.path.join(_wdir(root, wid), "workflow.json")
    meta = _read_json(p, {})
    meta.update(fields)
    _atomic_write(p, json.dumps(meta).encode())
    return meta


def _step_dir(root, wid, task_id):
    return os.path.join(_wdir(root, wid), "steps", task_id)


def _load_step(root, wid, task_id):
    p = os.path.join(_step_dir(root, wid, task_id), "output.pkl")
    if not os.path.exists(p):
        return False, None
    with open(p, "rb") as f:
        return True, cloudpickle.load(f)  # written by _commit_step below


def _commit_step(root, wid, task_id, value, meta):
    d = _step_dir(root, wid, task_id)
    _atomic_write(os.path.join(d, "output.pkl"), cloudpickle.dumps(value))
    _atomic_write(os.path.join(d, "meta.json"), json.dumps(meta, default=str).encode())


# ---------------------------------------------------------------------------- options
class options(dict):
    """``f.options(**workflow.options(task_id=..., checkpoint=..., catch_exceptions=...,
    metadata=...))`` or ``@workflow.options(...)`` above ``@ray.remote``."""

    _VALID = {"task_id", "metadata", "catch_exceptions", "checkpoint"}

    def __init__(self, **workflow_options):
        bad = set(workflow_options) - self._VALID
        if bad:
            raise ValueError(f"Invalid option keywords {bad} for workflow tasks. "
                             f"Valid ones are {self._VALID}.")
        super().__init__(_metadata={_META_KEY: dict(workflow_options)})

    def __call__(self, f):
        return f.options(**self)


def _wf_opts(node: FunctionNode) -> dict:
    return dict((node._bound_options.get("_metadata") or {}).get(_META_KEY) or {})


def _ray_opts(node: FunctionNode) -> dict:
    o = {k: v for k, v in node._bound_options.items() if k != "_metadata"}
    return o


# ---------------------------------------------------------------------------- special nodes
class _Continuation:
    def __init__(self, dag):
        self.dag = dag


def continuation(dag_node):
    """Return from a workflow step to continue with a sub-DAG (dynamic workflows)."""
    if not isinstance(dag_node, DAGNode):
        return dag_node
    return _Continuation(dag_node)


@ray.remote(num_cpus=0)
def _sleep_step(duration: float, deadline_file: str):
    try:
        with open(deadline_file) as f:
            deadline = float(f.read())
    except FileNotFoundError:
        deadline = time.time() + duration
        _atomic_write(deadline_file, str(deadline).encode())
    time.sleep(max(0.0, deadline - time.time()))
    return deadline


def sleep(duration: float) -> DAGNode:
    """A step that completes `duration` seconds after it first started — durably: a resumed
    workflow waits only for the remainder."""
    node = _sleep_step.options(**options(task_id=None)).bind(duration, None)
    node._wf_sleep = True
    return node


class EventListener:
    """Reference ``workflow/event_listener.py``: subclass and implement ``poll_for_event``
    (async) and optionally ``event_checkpointed``."""

    async def poll_for_event(self, *args, **kwargs):
        raise NotImplementedError

    async def event_checkpointed(self, event) -> None:
        pass


class TimerListener(EventListener):
    async def poll_for_event(self, timestamp):
        await asyncio.sleep(max(0.0, timestamp - time.time()))


class _EventResult:
    """An event step's value: _step checkpoints ``event`` first and only then tells the
    listener (``event_checkpointed``), so a provider never acknowledges an event the
    workflow could still lose (reference: workflow.wait_for_event semantics)."""

    def __init__(self, listener, event):
        self.listener, self.event = listener, event


@ray.remote(num_cpus=0)
def _event_step(listener_cls, args, kwargs):
    listener = listener_cls()
    return _EventResult(listener, asyncio.run(listener.poll_for_event(*args, **kwargs)))


# ------------------------------------------------------------------------ step context
def get_current_workflow_id() -> Optional[str]:
    """Inside a workflow step: the workflow's id (reference: workflow_context)."""
    from ray_amd.workflow import context

    return context.get_current_workflow_id()


def get_current_task_id() -> Optional[str]:
    """Inside a workflow step: the step's task id."""
    from ray_amd.workflow import context

    return context.get_current_task_id()


def wait_for_event(event_listener_type, *args, **kwargs) -> DAGNode:
    if not (isinstance(event_listener_type, type) and
            issubclass(event_listener_type, EventListener)):
        raise TypeError("event_listener_type must be a subclass of workflow.EventListener")
    return _event_step.bind(event_listener_type, args, kwargs)


# ---------------------------------------------------------------------------- execution
@ray.remote(max_retries=0)
def _step(fn, root, wid, task_id, wopts, cancel_file, *args, **kwargs):
    if os.path.exists(cancel_file):
        raise WorkflowCancellationError(wid)
    ok, value = _load_step(root, wid, task_id)
    if ok:
        return value
    t0 = time.time()
    catch = wopts.get("catch_exceptions", False)
    from ray_amd.workflow import context

    context._set(wid, task_id)
    evr = None
    try:
        out = fn(*args, **kwargs)
        evr = out if isinstance(out, _EventResult) else None
        if evr is not None:
            out = evr.event
        if isinstance(out, _Continuation):
            out = _execute(out.dag, root, wid, prefix=task_id + ".", inputs=((), {}),
                           cancel_file=cancel_file)
            out = ray.get(out)
        result = (out, None) if catch else out
    except WorkflowCancellationError:
        raise
    except Exception as e:  # noqa: BLE001
        if not catch:
            raise
        result = (None, e)
    if wopts.get("checkpoint", True):
        _commit_step(root, wid, task_id, result,
                     {"task_id": task_id, "task_options": wopts,
                      "user_metadata": wopts.get("metadata") or {},
                      "stats": {"start_time": t0, "end_time": time.time()}})
    if evr is not None:  # the event is durable now: let the listener acknowledge it
        asyncio.run(evr.listener.event_checkpointed(evr.event))
    return result


def _assign_task_ids(dag: DAGNode, prefix: str) -> Dict[str, str]:
    """Deterministic ids: explicit ``task_id`` or ``<fn name>`` with a DFS-order suffix."""
    ids: Dict[str, str] = {}
    used: Dict[str, int] = {}

    def visit(n):
        if n._stable_uuid in ids:
            return
        for c in n._children():
            visit(c)
        if isinstance(n, InputAttributeNode):
            visit(n._parent)
        if isinstance(n, FunctionNode):
            name = _wf_opts(n).get("task_id") or getattr(n._fn._function, "__name__", "task")
            k = used.get(name, 0)
            used[name] = k + 1
            ids[n._stable_uuid] = prefix + (name if k == 0 else f"{name}_{k}")

    visit(dag)
    return ids


def _execute(dag: DAGNode, root: str, wid: str, prefix: str, inputs, cancel_file: str):
    """Submit the DAG's steps; returns the ObjectRef (or value) of the root."""
    ids = _assign_task_ids(dag, prefix)
    cache: Dict[str, Any] = {}

    def resolve(v):
        if isinstance(v, DAGNode):
            return run_node(v)
        if isinstance(v, list):
            return [resolve(x) for x in v]
        if isinstance(v, tuple):
            return tuple(resolve(x) for x in v)
        if isinstance(v, dict):
            return {k: resolve(x) for k, x in v.items()}
        return v

    def run_node(n):
        key = n._stable_uuid
        if key in cache:
            return cache[key]
        if isinstance(n, (InputNode, InputAttributeNode)):
            out = n._exec({}, inputs)
        elif isinstance(n, MultiOutputNode):
            out = [resolve(x) for x in n._bound_args[0]]
        elif isinstance(n, FunctionNode):
            tid = ids[key]
            args = [resolve(a) for a in n._bound_args]
            kwargs = {k: resolve(v) for k, v in n._bound_kwargs.items()}
            if getattr(n, "_wf_sleep", False):
                args[1] = os.path.join(_step_dir(root, wid, tid), "deadline")
            ok, value = _load_step(root, wid, tid)
            if ok:
                out = value
            else:
                ro = _ray_opts(n)
                ro.setdefault("name", tid)
                out = _step.options(**ro).remote(n._fn._function, root, wid, tid, _wf_opts(n),
                                                 cancel_file, *args, **kwargs)
        else:
            raise TypeError(f"workflows support function DAG nodes only, got {type(n).__name__}")
        cache[key] = out
        return out

    return run_node(dag)


def _deep_get(v):
    if isinstance(v, ray.ObjectRef):
        return ray.get(v)
    if isinstance(v, list):
        return [_deep_get(x) for x in v]
    return v


@ray.remote(num_cpus=0, max_retries=0)
def _runner(root: str, wid: str):
    with open(os.path.join(_wdir(root, wid), "dag.pkl"), "rb") as f:
        dag, inputs = cloudpickle.load(f)  # written by _start below
    cancel_file = os.path.join(_wdir(root, wid), "CANCELED")
    _set_wf(root, wid, status=WorkflowStatus.RUNNING.value, runner_pid=os.getpid(),
            start_time=time.time())
    try:
        out = _deep_get(_execute(dag, root, wid, "", inputs, cancel_file))
    except Exception:
        if os.path.exists(cancel_file):
            _set_wf(root, wid, status=WorkflowStatus.CANCELED.value, end_time=time.time())
            raise WorkflowCancellationError(wid) from None
        _set_wf(root, wid, status=WorkflowStatus.FAILED.value, end_time=time.time())
        raise
    _atomic_write(os.path.join(_wdir(root, wid), "output.pkl"), cloudpickle.dumps(out))
    _set_wf(root, wid, status=WorkflowStatus.SUCCESSFUL.value, end_time=time.time())
    return out


_live_runs: Dict[str, Any] = {}


def _start(dag, args, kwargs, workflow_id, metadata) -> Tuple[str, Any]:
    root = _root()
    wid = workflow_id or f"workflow_{uuid.uuid4().hex[:12]}"
    d = _wdir(root, wid)
    meta = _read_json(os.path.join(d, "workflow.json"))
    if meta is not None:
        if meta.get("status") == WorkflowStatus.SUCCESSFUL.value:
            return wid, None  # already done: run() returns the stored output
    os.makedirs(d, exist_ok=True)
    if not os.path.exists(os.path.join(d, "dag.pkl")):
        _atomic_write(os.path.join(d, "dag.pkl"), cloudpickle.dumps((dag, (args, kwargs))))
    _set_wf(root, wid, status=WorkflowStatus.PENDING.value, user_metadata=metadata or {},
            created=time.time(), workflow_id=wid)
    ref = _runner.remote(root, wid)
    _live_runs[wid] = ref
    return wid, ref


def run(dag: DAGNode, *args, workflow_id: Optional[str] = None,
        metadata: Optional[Dict[str, Any]] = None, **kwargs) -> Any:
    """Run a workflow to completion and return its output."""
    return ray.get(run_async(dag, *args, workflow_id=workflow_id, metadata=metadata, **kwargs))


def run_async(dag: DAGNode, *args, workflow_id: Optional[str] = None,
              metadata: Optional[Dict[str, Any]] = None, **kwargs):
    if not isinstance(dag, DAGNode):
        raise TypeError("Input should be a DAG.")
    if metadata is not None and not isinstance(metadata, dict):
        raise ValueError("metadata must be a dict.")
    wid, ref = _start(dag, args, kwargs, workflow_id, metadata)
    return ref if ref is not None else ray.put(get_output(wid))


def resume(workflow_id: str) -> Any:
    return ray.get(resume_async(workflow_id))


def resume_async(workflow_id: str):
    root = _root()
    d = _wdir(root, workflow_id)
    meta = _read_json(os.path.join(d, "workflow.json"))
    if meta is None:
        raise WorkflowNotFoundError(workflow_id)
    if meta.get("status") == WorkflowStatus.CANCELED.value:
        raise WorkflowCancellationError(workflow_id)
    if meta.get("status") == WorkflowStatus.SUCCESSFUL.value:
        return ray.put(get_output(workflow_id))
    ref = _runner.remote(root, workflow_id)
    _live_runs[workflow_id] = ref
    return ref


def get_output(workflow_id: str, *, task_id: Optional[str] = None) -> Any:
    return ray.get(get_output_async(workflow_id, task_id=task_id))


def get_output_async(workflow_id: str, *, task_id: Optional[str] = None):
    root = _root()
    d = _wdir(root, workflow_id)
    if not os.path.isdir(d):
        raise WorkflowNotFoundError(workflow_id)
    if task_id is not None:
        ok, v = _load_step(root, workflow_id, task_id)
        if not ok:
            raise ValueError(f"task {task_id} of workflow {workflow_id} has no output yet")
        return ray.put(v)
    p = os.path.join(d, "output.pkl")
    if os.path.exists(p):
        with open(p, "rb") as f:
            return ray.put(cloudpickle.load(f))
    ref = _live_runs.get(workflow_id)
    if ref is not None:
        return ref
    st = get_status(workflow_id)
    if st in (WorkflowStatus.RUNNING, WorkflowStatus.PENDING):
        return _wait_output.remote(root, workflow_id)
    raise WorkflowExecutionError(workflow_id)


@ray.remote(num_cpus=0)
def _wait_output(root, wid):
    p = os.path.join(_wdir(root, wid), "output.pkl")
    while not os.path.exists(p):
        meta = _read_json(os.path.join(_wdir(root, wid), "workflow.json"), {})
        if meta.get("status") in (WorkflowStatus.FAILED.value, WorkflowStatus.CANCELED.value):
            raise WorkflowExecutionError(wid)
        time.sleep(0.1)
    with open(p, "rb") as f:
        return cloudpickle.load(f)


def _pid_alive(pid) -> bool:
    if not pid:
        return False
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


def get_status(workflow_id: str) -> WorkflowStatus:
    meta = _read_json(os.path.join(_wdir(_root(), workflow_id), "workflow.json"))
    if meta is None:
        raise WorkflowNotFoundError(workflow_id)
    st = WorkflowStatus(meta.get("status", "NONE"))
    if st == WorkflowStatus.RUNNING and not _pid_alive(meta.get("runner_pid")):
        return WorkflowStatus.RESUMABLE  # runner died (system failure): resumable
    return st


def list_all(status_filter=None) -> List[Tuple[str, WorkflowStatus]]:
    if isinstance(status_filter, (str, WorkflowStatus)):
        status_filter = {WorkflowStatus(status_filter)}
    elif status_filter is not None:
        status_filter = {WorkflowStatus(s) for s in status_filter}
    out = []
    root = _root()
    for wid in sorted(os.listdir(root)):
        if not os.path.exists(os.path.join(root, wid, "workflow.json")):
            continue
        st = get_status(wid)
        if status_filter is None or st in status_filter:
            out.append((wid, st))
    return out


def resume_all(include_failed: bool = False) -> List[Tuple[str, Any]]:
    want = {WorkflowStatus.RESUMABLE} | ({WorkflowStatus.FAILED} if include_failed else set())
    return [(wid, resume_async(wid)) for wid, st in list_all(want)]


def get_metadata(workflow_id: str, task_id: Optional[str] = None) -> Dict[str, Any]:
    root = _root()
    if task_id is None:
        meta = _read_json(os.path.join(_wdir(root, workflow_id), "workflow.json"))
        if meta is None:
            raise WorkflowNotFoundError(workflow_id)
        return {"status": get_status(workflow_id).value,
                "user_metadata": meta.get("user_metadata", {}),
                "stats": {"start_time": meta.get("start_time"),
                          "end_time": meta.get("end_time")}}
    m = _read_json(os.path.join(_step_dir(root, workflow_id, task_id), "meta.json"))
    if m is None:
        raise ValueError(f"No such task {task_id} in workflow {workflow_id}")
    return m


def cancel(workflow_id: str) -> None:
    root = _root()
    d = _wdir(root, workflow_id)
    if not os.path.isdir(d):
        raise WorkflowNotFoundError(workflow_id)
    _atomic_write(os.path.join(d, "CANCELED"), b"1")
    if get_status(workflow_id) not in (WorkflowStatus.SUCCESSFUL,):
        _set_wf(root, workflow_id, status=WorkflowStatus.CANCELED.value, end_time=time.time())
    ref = _live_runs.pop(workflow_id, None)
    if ref is not None:
        try:
            ray.cancel(ref, force=True)
        except Exception:
            pass


def delete(workflow_id: str) -> None:
    import shutil

    d = _wdir(_root(), workflow_id)
    if not os.path.isdir(d):
        raise WorkflowNotFoundError(workflow_id)
    if get_status(workflow_id) in WorkflowStatus.non_terminating_status():
        raise WorkflowError(f"Cannot delete running workflow {workflow_id}; cancel it first.")
    _live_runs.pop(workflow_id, None)
    shutil.rmtree(d, ignore_errors=True)
