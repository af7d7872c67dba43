"""``ray.util.client_connect`` (reference: python/ray/util/client_connect.py): connect the
process to a Ray Client server, the function form of ``ray_amd.init("ray://host:port")``
(util/client)."""

from __future__ import annotations

from typing import Any, Dict, Optional


def connect(conn_str: str, secure: bool = False, metadata=None,
            connection_retries: int = 3, job_config=None, namespace: Optional[str] = None,
            *, ignore_version: bool = False, _credentials=None,
            ray_init_kwargs: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    """Connect to ``host:port`` (or ``ray://host:port``); returns the connection info."""
    import ray_amd as ray

    if secure or _credentials is not None:
        raise NotImplementedError("TLS client connections are not supported")
    if ray.is_initialized():
        raise RuntimeError("ray_amd is already connected; call disconnect() first")
    addr = conn_str if conn_str.startswith("ray://") else f"ray://{conn_str}"
    kw = dict(ray_init_kwargs or {})
    if namespace is not None:
        kw["namespace"] = namespace
    if job_config is not None:
        kw["job_config"] = job_config
    ctx = ray.init(addr, **kw)
    info = {"num_clients": 1, "python_version": None, "ray_version": ray.__version__,
            "ray_commit": None, "protocol_version": None}
    if ctx is not None and hasattr(ctx, "address_info"):
        info.update(ctx.address_info if isinstance(ctx.address_info, dict) else {})
    return info


def disconnect():
    """Close the client connection (``ray_amd.shutdown()``)."""
    import ray_amd as ray

    ray.shutdown()
