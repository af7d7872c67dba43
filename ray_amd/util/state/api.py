"""State API: list / get / summarize cluster entities.

Parity with ``python/ray/util/state/api.py`` (list_actors:788, list_tasks:1020,
list_objects:1066, summarize_tasks:1382 ...) and the schemas of
``python/ray/util/state/common.py`` (ActorState:416, TaskState:~665, NodeState:496,
WorkerState:589, PlacementGroupState:467).

Design: the reference routes every query dashboard → GCS/raylets over gRPC. Here the
raylet (which also hosts the GCS tables) already holds every table in-process, so a
query is ONE request on the driver's existing raylet connection; filtering, limits and
summaries run client-side. Task states come from the task-event stream (owner:
PENDING_NODE_ASSIGNMENT / SUBMITTED_TO_WORKER; executor: RUNNING → FINISHED / FAILED)
merged per (task_id, attempt) in the raylet.
"""

from __future__ import annotations

import collections
import time
from typing import Any, Dict, List, Optional, Tuple

DEFAULT_LIMIT = 100
DEFAULT_RPC_TIMEOUT = 30


class RayStateApiException(Exception):
    pass


class StateRecord(dict):
    """A state row: dict access (``r["state"]``) and attribute access (``r.state``)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


class ActorState(StateRecord):
    pass


class TaskState(StateRecord):
    pass


class ObjectState(StateRecord):
    pass


class NodeState(StateRecord):
    pass


class WorkerState(StateRecord):
    pass


class PlacementGroupState(StateRecord):
    pass


class JobState(StateRecord):
    pass


class RuntimeEnvState(StateRecord):
    pass


_ACTOR_STATES = {0: "DEPENDENCIES_UNREADY", 1: "PENDING_CREATION", 2: "ALIVE", 3: "RESTARTING",
                 4: "DEAD"}


def _core(address=None):
    from ray_amd._private import worker as _w

    if address is not None and not _w.global_worker.connected:
        _w.init(address=address)
    return _w._check_connected()


def _match(row: dict, filters) -> bool:
    for key, pred, value in filters or ():
        have = row.get(key)
        if isinstance(have, str) and isinstance(value, str):
            eq = have.lower() == value.lower()
        else:
            eq = have == value or (have is not None and str(have) == str(value))
        if pred == "=" and not eq:
            return False
        if pred == "!=" and eq:
            return False
        if pred not in ("=", "!="):
            raise RayStateApiException(f"unsupported predicate {pred!r} (use '=' or '!=')")
    return True


def _finish(rows, cls, filters, limit):
    out = [cls(r) for r in rows if _match(r, filters)]
    return out[:limit] if limit is not None else out


# ---------------------------------------------------------------------------- sources
def _actor_rows(cw):
    rows = []
    for a in cw.call_raylet("list_actors"):
        st = a["state"]
        rows.append({
            "actor_id": a["actor_id"], "class_name": a["class_name"],
            "state": _ACTOR_STATES.get(st, st) if isinstance(st, int) else st,
            "job_id": a["job_id"].hex() if isinstance(a["job_id"], bytes) else a["job_id"],
            "name": a["name"], "namespace": a["namespace"], "node_id": a["node_id"],
            "pid": a["pid"], "ray_namespace": a["namespace"],
            "num_restarts": a["num_restarts"], "death_cause": a["death_cause"],
            "is_detached": a["lifetime"] == "detached",
            "required_resources": a["required_resources"],
            "start_time_ms": int(a["start_time"] * 1000) if a.get("start_time") else None,
            "end_time_ms": int(a["end_time"] * 1000) if a.get("end_time") else None,
        })
    return rows


def _task_rows(cw):
    cw._flush_task_events()
    time.sleep(0.02)
    return cw.call_raylet("list_tasks")


def _node_rows(cw):
    rows = []
    try:  # per-node telemetry (reporter.py): CPU / memory / per-GPU util, HBM, power, temp
        stats = cw.call_raylet("node_stats") or {}
    except Exception:  # noqa: BLE001
        stats = {}
    for n in cw.call_raylet("nodes"):
        rows.append({"node_id": n["NodeID"], "node_ip": n["NodeManagerAddress"],
                     "is_head_node": bool(n.get("is_head_node", True)),
                     "state": "ALIVE" if n["Alive"] else "DEAD",
                     "node_name": n["NodeManagerHostname"], "resources_total": n["Resources"],
                     "labels": n.get("Labels") or {},
                     "node_stats": stats.get(n["NodeID"])})
    return rows


def _worker_rows(cw):
    rows = []
    for w in cw.call_raylet("list_workers"):
        rows.append({"worker_id": w["worker_id"], "is_alive": w["state"] != "dead",
                     "worker_type": "DRIVER" if w["worker_type"] == "driver" else "WORKER",
                     "node_id": cw.node_id.hex(), "ip": "127.0.0.1", "pid": w["pid"],
                     "job_id": w["job_id"].hex() if isinstance(w["job_id"], bytes)
                     else w["job_id"], "actor_id": w["actor_id"], "gpu_ids": w["gpu_ids"],
                     "state": w["state"]})
    return rows


def _pg_rows(cw):
    rows = []
    for pid, p in (cw.call_raylet("pg_table", None) or {}).items():
        rows.append({"placement_group_id": pid.hex() if isinstance(pid, bytes) else pid,
                     "name": p["name"], "state": p["state"], "strategy": p["strategy"],
                     "bundles": [dict(b) for b in p["bundles"].values()],
                     "is_detached": False, "stats": p["stats"], "creator_job_id": None})
    return rows


def _job_rows(cw):
    rows = []
    for j in cw.call_raylet("list_jobs"):
        jid = j["job_id"]
        rows.append({"job_id": jid.hex() if isinstance(jid, bytes) else jid,
                     "status": j["status"], "driver_pid": j.get("driver_pid"),
                     "start_time": int(j["start_time"] * 1000),
                     "end_time": int(j["end_time"] * 1000) if j.get("end_time") else None,
                     "namespace": j.get("namespace"), "type": "DRIVER",
                     "metadata": j.get("metadata") or {},
                     "runtime_env": j.get("runtime_env") or {}})
    return rows


def _object_rows(cw):
    rows = []
    seen = set()
    for o in cw.call_raylet("list_objects"):
        seen.add(o["object_id"])
        rows.append({"object_id": o["object_id"], "object_size": o["object_size"],
                     "reference_type": "PINNED_IN_MEMORY" if o["pinned"] else "USED_BY_PENDING_TASK"
                     if o["ref_count"] else "LOCAL_REFERENCE", "node_id": o["node_id"],
                     "device": o.get("device"), "task_status": "FINISHED",
                     "pid": None, "ip": "127.0.0.1", "call_site": "disabled",
                     "type": "WORKER"})
    # the caller's own references to objects held inline (small objects never touch the store)
    with cw.lock:
        local = [(oid, e[0]) for oid, e in cw.refs.items()]
        owned = {oid: o for oid, o in cw.owned.items()}
    for oid, count in local:
        h = oid.hex()
        if h in seen:
            continue
        o = owned.get(oid)
        rows.append({"object_id": h, "object_size": (o.size if o is not None and o.size else
                                                     None),
                     "reference_type": "LOCAL_REFERENCE", "node_id": cw.node_id.hex(),
                     "device": "cpu", "task_status": "FINISHED" if o is None or o.ready
                     else "PENDING", "pid": None, "ip": "127.0.0.1", "call_site": "disabled",
                     "type": "DRIVER", "ref_count": count})
    return rows


# ---------------------------------------------------------------------------- list
def list_actors(address: Optional[str] = None, filters: Optional[List[Tuple[str, str, Any]]] = None,
                limit: int = DEFAULT_LIMIT, timeout: int = DEFAULT_RPC_TIMEOUT, detail: bool = False,
                raise_on_missing_output: bool = True, _explain: bool = False) -> List[ActorState]:
    return _finish(_actor_rows(_core(address)), ActorState, filters, limit)


def list_tasks(address=None, filters=None, limit=DEFAULT_LIMIT, timeout=DEFAULT_RPC_TIMEOUT,
               detail=False, raise_on_missing_output=True, _explain=False) -> List[TaskState]:
    return _finish(_task_rows(_core(address)), TaskState, filters, limit)


def list_objects(address=None, filters=None, limit=DEFAULT_LIMIT, timeout=DEFAULT_RPC_TIMEOUT,
                 detail=False, raise_on_missing_output=True, _explain=False) -> List[ObjectState]:
    return _finish(_object_rows(_core(address)), ObjectState, filters, limit)


def list_nodes(address=None, filters=None, limit=DEFAULT_LIMIT, timeout=DEFAULT_RPC_TIMEOUT,
               detail=False, raise_on_missing_output=True, _explain=False) -> List[NodeState]:
    return _finish(_node_rows(_core(address)), NodeState, filters, limit)


def list_workers(address=None, filters=None, limit=DEFAULT_LIMIT, timeout=DEFAULT_RPC_TIMEOUT,
                 detail=False, raise_on_missing_output=True, _explain=False) -> List[WorkerState]:
    return _finish(_worker_rows(_core(address)), WorkerState, filters, limit)


def list_placement_groups(address=None, filters=None, limit=DEFAULT_LIMIT,
                          timeout=DEFAULT_RPC_TIMEOUT, detail=False, raise_on_missing_output=True,
                          _explain=False) -> List[PlacementGroupState]:
    return _finish(_pg_rows(_core(address)), PlacementGroupState, filters, limit)


def list_jobs(address=None, filters=None, limit=DEFAULT_LIMIT, timeout=DEFAULT_RPC_TIMEOUT,
              detail=False, raise_on_missing_output=True, _explain=False) -> List[JobState]:
    return _finish(_job_rows(_core(address)), JobState, filters, limit)


def list_runtime_envs(address=None, filters=None, limit=DEFAULT_LIMIT, timeout=DEFAULT_RPC_TIMEOUT,
                      detail=False, raise_on_missing_output=True,
                      _explain=False) -> List[RuntimeEnvState]:
    cw = _core(address)
    envs = collections.Counter()
    for w in cw.call_raylet("list_workers"):
        envs[repr(w.get("runtime_env") or {})] += 1
    rows = [{"runtime_env": k, "success": True, "creation_time_ms": None, "ref_cnt": v,
             "node_id": cw.node_id.hex()} for k, v in envs.items()]
    return _finish(rows, RuntimeEnvState, filters, limit)


def list_cluster_events(address=None, filters=None, limit=DEFAULT_LIMIT, **kw) -> List[dict]:
    return []


# ---------------------------------------------------------------------------- get
def _get_one(rows, key, value, cls):
    for r in rows:
        if r.get(key) == value:
            return cls(r)
    return None


def get_actor(id: str, address=None, timeout=DEFAULT_RPC_TIMEOUT, _explain=False):
    return _get_one(_actor_rows(_core(address)), "actor_id", id, ActorState)


def get_task(id, address=None, timeout=DEFAULT_RPC_TIMEOUT, _explain=False):
    """All attempts of the task (the reference returns the latest attempt for a str id)."""
    rows = [r for r in _task_rows(_core(address)) if r["task_id"] == id]
    if not rows:
        return None
    return TaskState(max(rows, key=lambda r: r["attempt_number"]))


def get_node(id: str, address=None, timeout=DEFAULT_RPC_TIMEOUT, _explain=False):
    return _get_one(_node_rows(_core(address)), "node_id", id, NodeState)


def get_worker(id: str, address=None, timeout=DEFAULT_RPC_TIMEOUT, _explain=False):
    return _get_one(_worker_rows(_core(address)), "worker_id", id, WorkerState)


def get_placement_group(id: str, address=None, timeout=DEFAULT_RPC_TIMEOUT, _explain=False):
    return _get_one(_pg_rows(_core(address)), "placement_group_id", id, PlacementGroupState)


def get_job(id: str, address=None, timeout=DEFAULT_RPC_TIMEOUT, _explain=False):
    return _get_one(_job_rows(_core(address)), "job_id", id, JobState)


def get_objects(id: str, address=None, timeout=DEFAULT_RPC_TIMEOUT, _explain=False):
    return [ObjectState(r) for r in _object_rows(_core(address)) if r["object_id"] == id]


# ---------------------------------------------------------------------------- summarize
def summarize_tasks(address=None, timeout=DEFAULT_RPC_TIMEOUT, raise_on_missing_output=True,
                    _explain=False) -> Dict:
    """{"cluster": {"summary": {func_name: {"state_counts": {...}, "type": ...}},
    "total_tasks": n, ...}} (TaskSummaries in common.py)."""
    rows = _task_rows(_core(address))
    summary: Dict[str, dict] = {}
    for r in rows:
        s = summary.setdefault(r["func_or_class_name"], {
            "func_or_class_name": r["func_or_class_name"], "type": r["type"],
            "state_counts": collections.Counter()})
        s["state_counts"][r["state"]] += 1
    for s in summary.values():
        s["state_counts"] = dict(s["state_counts"])
    return {"cluster": {"summary": summary, "total_tasks": len(rows),
                        "total_actor_tasks": sum(r["type"] == "ACTOR_TASK" for r in rows),
                        "total_actor_scheduled": sum(r["type"] == "ACTOR_CREATION_TASK"
                                                     for r in rows),
                        "summary_by": "func_name"}}


def summarize_actors(address=None, timeout=DEFAULT_RPC_TIMEOUT, raise_on_missing_output=True,
                     _explain=False) -> Dict:
    rows = _actor_rows(_core(address))
    summary: Dict[str, dict] = {}
    for r in rows:
        s = summary.setdefault(r["class_name"], {"class_name": r["class_name"],
                                                 "state_counts": collections.Counter()})
        s["state_counts"][r["state"]] += 1
    for s in summary.values():
        s["state_counts"] = dict(s["state_counts"])
    return {"cluster": {"summary": summary, "total_actors": len(rows)}}


def summarize_objects(address=None, timeout=DEFAULT_RPC_TIMEOUT, raise_on_missing_output=True,
                      _explain=False) -> Dict:
    rows = _object_rows(_core(address))
    total = sum(r["object_size"] or 0 for r in rows)
    by_type = collections.Counter(r["reference_type"] for r in rows)
    return {"cluster": {"summary": {"disabled": {
        "total_objects": len(rows), "total_size_mb": total / 2 ** 20,
        "ref_type_counts": dict(by_type)}}, "total_objects": len(rows),
        "total_size_mb": total / 2 ** 20, "summary_by": "callsite"}}


class StateApiClient:
    """Thin object form of the module functions (reference: state_manager / StateApiClient)."""

    def __init__(self, address: Optional[str] = None):
        self.address = address

    @staticmethod
    def _name(resource) -> str:
        return str(getattr(resource, "value", resource)).lower()

    def list(self, resource, options=None, raise_on_missing_output=True,
             _explain=False, filters=None, limit=DEFAULT_LIMIT, **kw):
        """``resource``: a name or ``common.StateResource``; ``options``: a
        ``common.ListApiOptions`` (its filters / limit win over the keywords)."""
        if options is not None:
            filters, limit = options.filters, options.limit
        fn = {"actors": list_actors, "tasks": list_tasks, "objects": list_objects,
              "nodes": list_nodes, "workers": list_workers, "jobs": list_jobs,
              "placement_groups": list_placement_groups,
              "runtime_envs": list_runtime_envs,
              "cluster_events": list_cluster_events}[self._name(resource)]
        return fn(self.address, filters=filters, limit=limit)

    def get(self, resource, id: str, options=None, _explain=False):
        fn = {"actors": get_actor, "tasks": get_task, "objects": get_objects,
              "nodes": get_node, "workers": get_worker, "jobs": get_job,
              "placement_groups": get_placement_group}[self._name(resource)]
        return fn(id, self.address)

    def summary(self, resource, options=None, raise_on_missing_output=True, _explain=False,
                **kw):
        return {"tasks": summarize_tasks, "actors": summarize_actors,
                "objects": summarize_objects}[self._name(resource)](self.address)


# ---------------------------------------------------------------------------- logs
def _logs_dir(address=None):
    import os

    from ray_amd._private import worker as _w

    _core(address)
    return os.path.join(_w.global_worker.session_dir, "logs")


def list_logs(address=None, node_id=None, node_ip=None, glob_filter=None, timeout=None,
              **kw) -> dict:
    """{category: [file names]} of this node's session logs (reference: util/state/api.py
    list_logs); categories: worker_out, worker_err, other."""
    import fnmatch
    import os

    d = _logs_dir(address)
    out = {"worker_out": [], "worker_err": [], "other": []}
    for f in sorted(os.listdir(d)) if os.path.isdir(d) else []:
        if glob_filter and not fnmatch.fnmatch(f, glob_filter):
            continue
        cat = "worker_out" if f.startswith("worker-") and f.endswith(".out") else \
            "worker_err" if f.startswith("worker-") and f.endswith(".err") else "other"
        out[cat].append(f)
    return out


def get_log(address=None, node_id=None, node_ip=None, filename=None, actor_id=None,
            task_id=None, pid=None, follow=False, tail=-1, timeout=None, suffix="out",
            **kw):
    """Yield lines of one log file, chosen by ``filename``, or the worker ``pid`` (also
    resolved from ``actor_id``); ``tail`` > 0 keeps only the last lines; ``follow`` keeps
    yielding appended lines."""
    import glob
    import os
    import time

    d = _logs_dir(address)
    if filename is None:
        if pid is None and actor_id is not None:
            a = get_actor(actor_id, address=address)
            pid = getattr(a, "pid", None) if a is not None else None
        if pid is None:
            raise ValueError("get_log needs filename, pid or actor_id")
        hits = glob.glob(os.path.join(d, f"worker-*-{pid}.{suffix}"))
        if not hits:
            raise FileNotFoundError(f"no {suffix} log for pid {pid} in {d}")
        path = hits[0]
    else:
        path = os.path.join(d, filename)
    with open(path, "r", errors="replace") as f:
        lines = f.readlines()
        for ln in (lines[-tail:] if tail and tail > 0 else lines):
            yield ln.rstrip("\n")
        while follow:
            ln = f.readline()
            if ln:
                yield ln.rstrip("\n")
            else:
                time.sleep(0.2)
