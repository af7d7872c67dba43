"""ray_amd — an MI355X-native distributed ML runtime with Ray's API surface.

    import ray_amd as ray
    ray.init()

    @ray.remote
    def f(x): return x * 2

    ray.get([f.remote(i) for i in range(4)])

Compute path: PyTorch-ROCm + hand-written HIP/CDNA4 kernels (ray_amd.ops) +
RCCL over xGMI (ray_amd.util.collective, ray_amd.parallel). Runtime core:
native C++ (ray_amd._native: shared-memory object store, frame I/O loop,
resource scheduler).
"""

from __future__ import annotations

import os as _os

# 8 hardware queues per process (RAY_AMD_HW_QUEUES; see _private/worker_main.py)
if _os.environ.get("RAY_AMD_HW_QUEUES", "8") != "0":  # 0: leave HIP's setting alone
    _os.environ["GPU_MAX_HW_QUEUES"] = _os.environ.get("RAY_AMD_HW_QUEUES", "8")

__version__ = "0.1.0"

from ray_amd._private.worker import (LOCAL_MODE, SCRIPT_MODE, WORKER_MODE,  # noqa: F401
                                     available_resources, cancel, cluster_resources, get,
                                     get_actor, get_gpu_ids, init, is_initialized, kill, method,
                                     nodes, put, shutdown, timeline, wait)
from ray_amd.actor import ActorClass, ActorHandle  # noqa: F401
from ray_amd.object_ref import (DynamicObjectRefGenerator, ObjectRef,  # noqa: F401
                                ObjectRefGenerator)
from ray_amd._private.ids import (ActorClassID, ActorID, FunctionID, JobID,  # noqa: F401
                                  NodeID, ObjectID, PlacementGroupID, TaskID, UniqueID,
                                  WorkerID)
from ray_amd.remote_function import RemoteFunction  # noqa: F401
from ray_amd.runtime_context import get_runtime_context  # noqa: F401
from ray_amd import exceptions  # noqa: F401
from ray_amd import internal  # noqa: F401


def remote(*args, **kwargs):
    """Decorator for remote functions and actor classes (parity: ray.remote)."""
    import inspect

    def make(obj, options):
        if inspect.isclass(obj):
            return ActorClass(obj, options)
        if callable(obj):
            return RemoteFunction(obj, options)
        raise TypeError("The @ray_amd.remote decorator must be applied to either a function "
                        "or a class.")

    if len(args) == 1 and not kwargs and callable(args[0]):
        return make(args[0], {})
    if args:
        raise TypeError("The @ray_amd.remote decorator must be applied either with no arguments "
                        "and no parentheses, or with keyword arguments only.")
    return lambda obj: make(obj, kwargs)


def java_function(*a, **k):
    raise NotImplementedError("cross-language calls are not supported by ray_amd")


java_actor_class = cpp_function = java_function


class Language:
    PYTHON = "PYTHON"


__all__ = [
    "__version__", "available_resources", "cancel", "cluster_resources", "get", "get_actor",
    "get_gpu_ids", "init", "is_initialized", "kill", "method", "nodes", "put", "remote",
    "shutdown", "timeline", "wait", "get_runtime_context", "ObjectRef", "ObjectRefGenerator",
    "ActorHandle", "LOCAL_MODE", "SCRIPT_MODE", "WORKER_MODE", "exceptions", "Language",
    "client", "ClientBuilder", "show_in_dashboard", "DynamicObjectRefGenerator",
    "ActorClassID", "ActorID", "NodeID", "JobID", "WorkerID", "FunctionID", "ObjectID",
    "TaskID", "UniqueID", "PlacementGroupID", "internal",
]

from ray_amd.client_builder import ClientBuilder, client  # noqa: F401,E402


def show_in_dashboard(message: str, key: str = "", dtype: str = "text"):
    """Attach a message to the current actor / task, shown by the dashboard and the state
    API (``list_actors(detail=True)``) (reference: python/ray/_private/worker.py)."""
    if dtype not in ("text", "html"):
        raise ValueError(f"dtype accepts only text or html, got {dtype!r}")
    from ray_amd._private import worker as _w

    cw = _w._check_connected()
    msgs = getattr(cw, "dashboard_messages", None)
    if msgs is None:
        msgs = cw.dashboard_messages = {}
    msgs[key] = {"message": message, "dtype": dtype}


_LAZY_SUBPACKAGES = ("data", "train", "tune", "serve", "rllib", "util", "workflow", "dag",
                     "air", "cluster_utils", "job_submission", "dashboard", "experimental",
                     "autoscaler", "runtime_env")


def __getattr__(name):
    # `import ray_amd; ray_amd.data.range(...)` without importing heavy subpackages up
    # front (reference: python/ray/__init__.py module __getattr__)
    if name in _LAZY_SUBPACKAGES:
        import importlib

        return importlib.import_module(f"ray_amd.{name}")
    raise AttributeError(f"module 'ray_amd' has no attribute {name!r}")
