"""debugpy-based remote debugging of tasks and actors (reference:
python/ray/util/ray_debugpy.py). ``set_trace()`` opens a debugpy listener in the worker
and waits for an IDE to attach; the post-mortem hook does the same on an exception. Needs
the ``debugpy`` package; without it, use ``ray_amd.util.pdb.set_trace`` (the rpdb-based
debugger with the ``debug`` CLI), which this framework ships."""

from __future__ import annotations

import os
import socket

DEBUGPY_PORT_ENV = "RAY_DEBUGPY_PORT"


def _debugpy():
    try:
        import debugpy

        return debugpy
    except ImportError:
        raise ImportError("ray_debugpy requires debugpy (`pip install debugpy`); "
                          "ray_amd.util.pdb.set_trace() needs nothing extra") from None


def _listen(debugpy):
    port = int(os.environ.get(DEBUGPY_PORT_ENV, "0"))
    if not port:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
    host, port = debugpy.listen(("127.0.0.1", port))
    print(f"[ray_amd] debugpy listening on {host}:{port}; attach your IDE", flush=True)
    return port


def set_trace(breakpoint_uuid=None):
    """Break into debugpy inside a task or actor method."""
    dbg = _debugpy()
    if not dbg.is_client_connected():
        _listen(dbg)
        dbg.wait_for_client()
    dbg.breakpoint()


def _post_mortem():
    dbg = _debugpy()
    if not dbg.is_client_connected():
        _listen(dbg)
        dbg.wait_for_client()
    import sys

    dbg.breakpoint()
    return sys.exc_info()


def _is_ray_debugger_post_mortem_enabled() -> bool:
    return os.environ.get("RAY_DEBUG_POST_MORTEM", "0") == "1"
