"""ray_amd.util (reference: python/ray/util/__init__.py)."""

from ray_amd._private.serialization import (deregister_serializer,  # noqa: F401
                                            register_serializer)
from ray_amd.util import iter  # noqa: F401,A004
from ray_amd.util import ray_debugpy  # noqa: F401
from ray_amd.util.actor_group import ActorGroup  # noqa: F401
from ray_amd.util.actor_pool import ActorPool  # noqa: F401
from ray_amd.util.debug import (disable_log_once_globally,  # noqa: F401
                                enable_periodic_logging, log_once)
from ray_amd.util.placement_group import (get_current_placement_group,  # noqa: F401
                                          get_placement_group, placement_group,
                                          placement_group_table, remove_placement_group)


def get_node_ip_address():
    """This node's address as registered with the cluster (RAY_AMD_NODE_IP on the node,
    else 127.0.0.1 for a single-machine cluster)."""
    import os

    from ray_amd._private import worker as W

    cw = W.global_worker.core
    ip = getattr(cw, "node_ip", None) if cw is not None else None
    return ip or os.environ.get("RAY_AMD_NODE_IP", "127.0.0.1")


def list_named_actors(all_namespaces: bool = False):
    from ray_amd._private import worker as W

    cw = W._check_connected()
    return cw.call_raylet("list_named_actors", all_namespaces, cw.namespace)


def inspect_serializability(obj, name=None, depth=3, print_file=None):
    import cloudpickle

    try:
        cloudpickle.dumps(obj)
        return True, set()
    except Exception as e:  # noqa: BLE001
        return False, {repr(e)}


__all__ = ["ActorPool", "ActorGroup", "iter", "placement_group", "placement_group_table", "get_placement_group",
           "remove_placement_group", "get_current_placement_group", "register_serializer",
           "deregister_serializer", "get_node_ip_address", "list_named_actors",
           "inspect_serializability"]


def __getattr__(name):
    # heavier submodules on first use: ray_amd.util.collective / accelerators / pdb
    if name in ("collective", "accelerators", "pdb", "rpdb", "joblib", "state", "metrics",
                "queue", "multiprocessing", "scheduling_strategies", "annotations", "timer"):
        import importlib

        return importlib.import_module(f"ray_amd.util.{name}")
    raise AttributeError(f"module 'ray_amd.util' has no attribute {name!r}")


def connect(conn_str: str, secure: bool = False, metadata=None, connection_retries: int = 3,
            job_config=None, namespace: str | None = None, **kw):
    """Legacy Ray Client entry (reference: util/client_connect.py): ``connect("host:port")``."""
    import ray_amd

    addr = conn_str if conn_str.startswith("ray://") else "ray://" + conn_str
    ray_amd.init(address=addr, namespace=namespace)
    return {"num_clients": 1, "ray_version": ray_amd.__version__}


def disconnect():
    import ray_amd

    ray_amd.shutdown()
