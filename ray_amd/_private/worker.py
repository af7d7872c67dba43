"""Global worker state and the core public API (reference: python/ray/_private/worker.py).

``init`` starts (or attaches to) a node: it launches the raylet process, which
creates the shared-memory object store and the worker pool, then connects this
process as the job's driver.
"""

from __future__ import annotations

import atexit
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

from ray_amd.exceptions import GetTimeoutError, RaySystemError

SCRIPT_MODE = 0
WORKER_MODE = 1
LOCAL_MODE = 2

ROOT_TMP = os.environ.get("RAY_AMD_TMPDIR", os.path.join(tempfile.gettempdir(), "ray_amd_sessions"))
CURRENT_CLUSTER_FILE = os.path.join(ROOT_TMP, "ray_current_cluster")


class Worker:
    def __init__(self):
        self.core = None
        self.mode = None
        self.raylet_proc = None
        self.session_dir = None
        self.node_started_here = False
        self.lock = threading.RLock()
        self.namespace = None
        self.runtime_env = None
        self.job_config = None
        self._local_mode = False
        self.dashboard_proc = None
        self.dashboard_url = None

    @property
    def connected(self):
        return self.core is not None

    def connect_worker(self, cw):
        self.core = cw
        self.mode = WORKER_MODE
        self.session_dir = cw.session_dir


global_worker = Worker()
_global_node_lock = threading.Lock()


def is_initialized() -> bool:
    return global_worker.connected


def _default_object_store_memory():
    try:
        st = os.statvfs("/dev/shm")
        shm_free = st.f_bavail * st.f_frsize
    except OSError:
        shm_free = 4 << 30
    total = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES")
    return int(max(256 << 20, min(0.3 * total, 0.8 * shm_free, 200 << 30)))


# _system_config keys this runtime honours, as the RAY_<key> variables the raylet reads
# (reference names: memory monitor and worker-killing policy)
SYSTEM_CONFIG_KEYS = ("memory_usage_threshold", "memory_monitor_refresh_ms",
                      "min_memory_free_bytes", "worker_killing_policy")


def _node_env(system_config, log_to_driver, logging_level) -> dict:
    env = {}
    for k, v in (system_config or {}).items():
        if k not in SYSTEM_CONFIG_KEYS:
            raise ValueError(f"unsupported _system_config key {k!r}; supported: "
                             f"{list(SYSTEM_CONFIG_KEYS)}")
        env[f"RAY_{k}"] = str(v)
    if not log_to_driver:
        env["RAY_AMD_LOG_TO_DRIVER"] = "0"  # worker output only in <session>/logs
    if logging_level is not None:
        env["RAY_AMD_LOGGING_LEVEL"] = str(logging_level)
    return env


def _configure_logging(level, fmt):
    """init(logging_level=..., logging_format=...): the ray_amd logger's level and format in
    this driver (workers get the level through RAY_AMD_LOGGING_LEVEL)."""
    import logging

    lg = logging.getLogger("ray_amd")
    if level is not None:
        lg.setLevel(level if isinstance(level, int) else str(level).upper())
    if fmt is not None:
        h = logging.StreamHandler()
        h.setFormatter(logging.Formatter(fmt))
        lg.handlers = [h]
        lg.propagate = False


def _start_raylet(session_dir, num_cpus, num_gpus, resources, object_store_memory, labels,
                  head=True, detach_output=False, extra_env=None):
    os.makedirs(session_dir, exist_ok=True)
    store_path = "/dev/shm/ray_amd_" + os.path.basename(session_dir)
    cmd = [sys.executable, "-m", "ray_amd._private.raylet", "--session-dir", session_dir,
           "--store-path", store_path, "--object-store-memory", str(object_store_memory),
           "--resources", json.dumps(resources or {}), "--labels", json.dumps(labels or {})]
    if num_cpus is not None:
        cmd += ["--num-cpus", str(int(num_cpus))]
    if num_gpus is not None:
        cmd += ["--num-gpus", str(int(num_gpus))]
    if head:
        cmd.append("--head")
    if not detach_output:
        # fate sharing (reference: services.py start_ray_process(fate_share=True)): a node
        # started by ray.init() / cluster_utils exits when this process is gone, even if it
        # was killed without running ray.shutdown(); `start` (detached) nodes outlive it
        cmd += ["--fate-share-pid", str(os.getpid())]
    env = dict(os.environ)
    env.update(extra_env or {})
    pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH")
                                    else "")
    out = None
    if detach_output:  # a daemonised node (CLI `start`) must not hold the caller's stdout
        out = open(os.path.join(session_dir, "raylet.out"), "ab")
    proc = subprocess.Popen(cmd, env=env, close_fds=True, start_new_session=True, stdout=out,
                            stderr=subprocess.STDOUT if out else None,
                            stdin=subprocess.DEVNULL if out else None)
    ready = os.path.join(session_dir, "raylet.ready")
    t0 = time.time()
    while not os.path.exists(ready):
        if proc.poll() is not None:
            raise RaySystemError(RuntimeError(f"raylet exited with code {proc.returncode}"))
        if time.time() - t0 > 120:
            proc.kill()
            raise RaySystemError(RuntimeError("timed out waiting for the raylet"))
        time.sleep(0.01)
    with open(ready) as f:
        info = json.load(f)
    return proc, info["addr"]


def new_session_dir():
    os.makedirs(ROOT_TMP, exist_ok=True)
    ts = time.strftime("%Y-%m-%d_%H-%M-%S")
    return os.path.join(ROOT_TMP, f"session_{ts}_{os.getpid()}_{os.urandom(3).hex()}")


def init(address: str | None = None, *, num_cpus=None, num_gpus=None, resources=None,
         labels=None, object_store_memory=None, local_mode=False, ignore_reinit_error=False,
         include_dashboard=None, dashboard_host=None, dashboard_port=None, job_config=None,
         configure_logging=True, logging_level=None, logging_format=None, log_to_driver=True,
         namespace=None, runtime_env=None, _temp_dir=None, _system_config=None,
         storage=None, **kwargs):
    """Start or connect to a ray_amd node (parity: ray.init)."""
    from .core_worker import CoreWorker
    from .ids import random_bytes

    unknown = sorted(k for k in kwargs if not k.startswith("_"))
    if unknown:
        raise TypeError(f"init() got unexpected keyword argument(s) {unknown}")
    hook = kwargs.pop("_tracing_startup_hook", None)
    if hook:  # "module:fn" (or "module.fn"): enables span export in this process
        import importlib

        mod, _, fn = hook.partition(":") if ":" in hook else hook.rpartition(".")
        getattr(importlib.import_module(mod), fn)()
    for k in kwargs:  # private reference knobs with no meaning here (_redis_password, ...)
        import warnings

        warnings.warn(f"ray_amd.init: internal option {k} has no effect", stacklevel=2)
    if configure_logging:
        _configure_logging(logging_level, logging_format)
    node_env = _node_env(_system_config, log_to_driver, logging_level)
    if storage is not None:
        # default storage of Train / Tune / Workflow results (RunConfig.storage_path)
        os.environ["RAY_AMD_STORAGE"] = str(storage)

    if job_config is not None:
        namespace = namespace or job_config.ray_namespace
        if runtime_env is None and job_config.runtime_env:
            runtime_env = dict(job_config.runtime_env)
    with _global_node_lock:
        if global_worker.connected:
            if ignore_reinit_error:
                return RayContext(global_worker)
            raise RuntimeError("Maybe you called ray_amd.init twice by accident? Use "
                               "ignore_reinit_error=True to ignore this.")
        if address is None:
            address = os.environ.get("RAY_ADDRESS") or os.environ.get("RAY_AMD_ADDRESS")
        if address and address.startswith("ray://"):
            # Ray Client mode: every API call is forwarded to a client server
            from ray_amd.util.client import DEFAULT_PORT, ClientCoreWorker

            hp = address[len("ray://"):]
            host, _, port = hp.partition(":")
            cw = ClientCoreWorker(host or "127.0.0.1", int(port or DEFAULT_PORT), namespace,
                                  runtime_env)
            global_worker.core = cw
            global_worker.mode = SCRIPT_MODE
            global_worker.session_dir = address
            global_worker.namespace = cw.namespace
            global_worker.node_started_here = False
            atexit.register(shutdown)
            return RayContext(global_worker)
        if address in (None, "local", ""):
            from . import shm_segment

            shm_segment.sweep_dead()  # named segments of dead sessions (RAY_AMD_SHM_MEMFD=0)
            session = new_session_dir() if _temp_dir is None else os.path.join(
                _temp_dir, os.path.basename(new_session_dir()))
            osm = int(object_store_memory or _default_object_store_memory())
            proc, raylet_addr = _start_raylet(session, num_cpus, num_gpus, resources, osm,
                                              labels, extra_env=node_env)
            global_worker.raylet_proc = proc
            global_worker.node_started_here = True
            if include_dashboard:
                from ray_amd.dashboard import start_dashboard

                global_worker.dashboard_proc, global_worker.dashboard_url = start_dashboard(
                    session, dashboard_host or "127.0.0.1", int(dashboard_port or 8265))
        else:
            if _system_config:
                raise ValueError("_system_config applies when init() starts a new node, not "
                                 "when connecting to an existing cluster")
            if address == "auto":
                if not os.path.exists(CURRENT_CLUSTER_FILE):
                    raise ConnectionError("Could not find any running ray_amd instance. "
                                          "Start one with `python -m ray_amd.scripts start "
                                          "--head`.")
                with open(CURRENT_CLUSTER_FILE) as f:
                    session = f.read().strip()
            else:
                session = address
            raylet_addr = os.path.join(session, "sockets", "raylet.sock")
            global_worker.node_started_here = False
        cw = CoreWorker(mode="driver", session_dir=session, raylet_addr=raylet_addr,
                        worker_id=random_bytes(16), namespace=namespace)
        cw.local_mode = bool(local_mode)
        global_worker.core = cw
        global_worker.mode = LOCAL_MODE if local_mode else SCRIPT_MODE
        global_worker.session_dir = session
        global_worker.namespace = cw.namespace
        global_worker.runtime_env = runtime_env
        global_worker.job_config = job_config
        sp = [os.path.abspath(p) if p else os.getcwd() for p in sys.path]
        main = sys.modules.get("__main__")
        if main is not None and getattr(main, "__file__", None):
            sp.insert(0, os.path.dirname(os.path.abspath(main.__file__)))
        sp.insert(0, os.getcwd())
        runtime_env = cw._export_renv(runtime_env)
        global_worker.runtime_env = runtime_env
        if job_config is not None:
            # code_search_path: importable in every worker of the job (first on the path)
            sp = list(job_config.code_search_path) + sp
            for p in reversed(job_config.code_search_path):
                if p not in sys.path:
                    sys.path.insert(0, p)
            cw.call_raylet("set_job_info", cw.job_id, sp, runtime_env,
                           job_config._to_dict())
        else:
            cw.call_raylet("set_job_info", cw.job_id, sp, runtime_env)
        atexit.register(shutdown)
        return RayContext(global_worker)


class RayContext(dict):
    def __init__(self, w):
        super().__init__(address=w.session_dir, session_dir=w.session_dir,
                         node_id=w.core.node_id.hex() if w.core else None,
                         namespace=w.namespace)
        self.address_info = dict(self)
        self.dashboard_url = w.dashboard_url

    def __enter__(self):
        return self

    def __exit__(self, *a):
        shutdown()

    def disconnect(self):
        shutdown()


def shutdown(_exiting_interpreter=False):
    w = global_worker
    dx = sys.modules.get("ray_amd.data._executor")
    if dx is not None and w.core is not None:  # abandoned Data iterators stop first
        try:
            dx.stop_all()
        except Exception:  # noqa: BLE001
            pass
    with _global_node_lock:
        cw = w.core
        if cw is None:
            return
        try:
            if w.dashboard_proc is not None:
                w.dashboard_proc.terminate()
                try:
                    w.dashboard_proc.wait(timeout=5)
                except Exception:
                    w.dashboard_proc.kill()
                w.dashboard_proc = None
                w.dashboard_url = None
            if w.node_started_here:
                try:
                    cw.call_raylet("shutdown", timeout=5)
                except Exception:
                    pass
        finally:
            cw.shutdown()
            w.core = None
            if w.raylet_proc is not None:
                try:
                    w.raylet_proc.wait(timeout=10)
                except Exception:
                    w.raylet_proc.kill()
                w.raylet_proc = None
        _reset_module_state()


def _reset_module_state():
    try:
        from ray_amd import actor as _actor

        _actor._reset()
    except Exception:
        pass


def _check_connected():
    if not global_worker.connected:
        # auto-init (reference: auto_init_hook)
        init()
    return global_worker.core


def put(value, *, _owner=None):
    from ray_amd.object_ref import ObjectRef

    cw = _check_connected()
    if isinstance(value, ObjectRef):
        raise TypeError("Calling 'put' on an ObjectRef is not allowed.")
    return cw.put_object(value)


def get(object_refs, *, timeout=None):
    from ray_amd.object_ref import ObjectRef, ObjectRefGenerator

    cw = _check_connected()
    if isinstance(object_refs, ObjectRefGenerator):
        object_refs = list(object_refs)
    cd = _compiled_dag_get(object_refs, timeout)
    if cd is not None:
        return cd[0]
    single = isinstance(object_refs, ObjectRef)
    if single:
        refs = [object_refs]
    elif isinstance(object_refs, (list, tuple)):
        refs = list(object_refs)
        for r in refs:
            if not isinstance(r, ObjectRef):
                raise TypeError(f"ray_amd.get() expects ObjectRef or list of ObjectRefs, got "
                                f"{type(r)}")
    else:
        raise ValueError(f"Invalid type of object refs, {type(object_refs)}, is given. "
                         "'object_refs' must either be an ObjectRef or a list of ObjectRefs.")
    if timeout is not None and timeout < 0:
        raise ValueError("timeout must be >= 0")
    vals = cw.get_objects(refs, timeout)
    return vals[0] if single else vals


def _compiled_dag_get(refs, timeout):
    """ray.get on CompiledDAGRef(s): resolved through the DAG's output channels."""
    import sys

    m = sys.modules.get("ray_amd.dag.compiled_dag_node")
    if m is None:
        return None
    R = m.CompiledDAGRef
    if isinstance(refs, R):
        return (refs.get(timeout),)
    if isinstance(refs, (list, tuple)) and refs and all(isinstance(r, R) for r in refs):
        return ([r.get(timeout) for r in refs],)
    return None


_ref_id = __import__("operator").attrgetter("_id")


def wait(object_refs, *, num_returns=1, timeout=None, fetch_local=True):
    from ray_amd.object_ref import ObjectRef

    cw = _check_connected()
    if isinstance(object_refs, ObjectRef):
        raise TypeError("wait() expected a list of ray_amd.ObjectRef, got a single ObjectRef")
    refs = list(object_refs)
    ids = list(map(_ref_id, refs))
    idset = set(ids)
    if len(idset) != len(ids):
        raise ValueError("Wait requires a list of unique object refs.")
    if num_returns <= 0 or num_returns > len(refs):
        raise ValueError("Invalid number of objects to return %d." % num_returns)
    ready = cw.wait_refs(idset, num_returns, timeout)
    if len(ready) * 8 < len(ids):
        # few ready refs (the common one-at-a-time loop): locate them with C-level index
        # scans and cut the not-ready list out of the input by slicing
        pos = sorted(ids.index(i) for i in ready)[:num_returns]
        r_list = [refs[i] for i in pos]
        nr, prev = [], 0
        for i in pos:
            nr += refs[prev:i]
            prev = i + 1
        nr += refs[prev:]
        return r_list, nr
    if len(ready) > num_returns:  # keep the first ready ones in input order
        ready = set([i for i in ids if i in ready][:num_returns])
    r_list = [r for r, i in zip(refs, ids) if i in ready]
    nr = [r for r, i in zip(refs, ids) if i not in ready]
    return r_list, nr


def kill(actor, *, no_restart=True):
    from ray_amd.actor import ActorHandle

    if not isinstance(actor, ActorHandle):
        raise ValueError(f"ray_amd.kill() only supported for actors. Got: {type(actor)}.")
    cw = _check_connected()
    cw.kill_actor(actor._actor_id, no_restart)


def cancel(object_ref, *, force=False, recursive=True):
    from ray_amd.object_ref import ObjectRef

    cw = _check_connected()
    if not isinstance(object_ref, ObjectRef):
        raise TypeError("ray_amd.cancel() only supported for ObjectRefs")
    cw.cancel(object_ref, force, recursive)


def get_actor(name: str, namespace: str | None = None):
    from ray_amd.actor import ActorHandle

    cw = _check_connected()
    ns = namespace or cw.namespace
    info = cw.call_raylet("get_named_actor", name, ns)
    if info is None:
        raise ValueError(f"Failed to look up actor with name '{name}'. This could because 1. "
                         "You are trying to look up a named actor you didn't create. 2. The "
                         "named actor died. 3. You did not use a namespace matching the "
                         "namespace of the actor.")
    return ActorHandle._from_info(info["actor_id"], info["class_name"], info["method_meta"],
                                  info["owner"])


def cluster_resources():
    return _check_connected().call_raylet("cluster_resources")


def available_resources():
    return _check_connected().call_raylet("available_resources")


def nodes():
    return _check_connected().call_raylet("nodes")


def get_gpu_ids():
    cw = _check_connected()
    return list(cw.gpu_ids)


def timeline(filename=None):
    """Chrome-trace of task execution (reference: ray.timeline)."""
    cw = _check_connected()
    cw._flush_task_events()
    time.sleep(0.05)
    events = cw.call_raylet("get_task_events")
    trace = []
    for ev in events:
        tid, name, t0, t1, pid, actor_id, status = ev[:7]
        trace.append({"cat": "task", "name": name, "ph": "X", "pid": pid, "tid": pid,
                      "ts": t0 * 1e6, "dur": (t1 - t0) * 1e6,
                      "args": {"task_id": tid.hex(), "status": status,
                               "actor_id": actor_id.hex() if actor_id else None}})
    if filename:
        with open(filename, "w") as f:
            json.dump(trace, f)
        return None
    return trace


def method(*args, **kwargs):
    """@ray.method decorator: per-method options (num_returns, concurrency_group...)."""

    def deco(m):
        m.__ray_amd_method_options__ = kwargs
        return m

    if len(args) == 1 and callable(args[0]) and not kwargs:
        return deco(args[0])
    return deco


GetTimeoutError  # noqa: B018
