"""Remote pdb for tasks and actors: ``ray_amd.util.pdb.set_trace()`` / ``ray_amd debug``.

Reference parity: python/ray/util/rpdb.py:278 (set_trace), :326 (post-mortem), :340
(client). A breakpoint in a worker opens a TCP listener on the node's address, publishes
``{host, port, pid, task}`` in the internal KV under ``RAY_PDB_<uuid>`` and blocks until a
client attaches; ``ray_amd debug`` (scripts) lists the live breakpoints and connects the
terminal to one. In the driver, set_trace falls back to the local pdb.
"""

from __future__ import annotations

import json
import os
import pdb
import socket
import sys
import uuid

_PREFIX = "RAY_PDB_"
_NS = "_ray_amd_debug"


class _SockIO:
    """Line-oriented text file over a socket (pdb's stdin / stdout)."""

    def __init__(self, conn):
        self._conn = conn
        self._r = conn.makefile("r", encoding="utf-8", newline="\n")

    def readline(self, *a):
        return self._r.readline()

    def write(self, data):
        self._conn.sendall(data.replace("\n", "\r\n").encode())
        return len(data)

    def flush(self):
        pass

    def close(self):
        try:
            self._r.close()
        finally:
            self._conn.close()


class RemotePdb(pdb.Pdb):
    """pdb served over one TCP connection; detaches on continue / quit."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, *, key: str | None = None,
                 quiet: bool = False):
        self._listener = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._listener.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._listener.bind((host, port))
        self._listener.listen(1)
        self.host, self.port = self._listener.getsockname()
        self.key = key
        if not quiet:
            print(f"RemotePdb session open at {self.host}:{self.port} (pid {os.getpid()}); "
                  "attach with `python -m ray_amd.scripts.scripts debug`", file=sys.__stderr__,
                  flush=True)
        self._io = None

    def listen(self):
        conn, _ = self._listener.accept()
        self._listener.close()
        self._io = _SockIO(conn)
        super().__init__(stdin=self._io, stdout=self._io, skip=["ray_amd.*"])
        self.use_rawinput = False
        self.prompt = "(ray-pdb) "

    def _detach(self):
        _unregister(self.key)
        if self._io is not None:
            try:
                self._io.close()
            except OSError:
                pass
            self._io = None

    def do_continue(self, arg):
        r = super().do_continue(arg)
        self._detach()
        return r

    do_c = do_cont = do_continue

    def do_quit(self, arg):
        r = super().do_quit(arg)
        self._detach()
        return r

    do_q = do_exit = do_quit

    def do_EOF(self, arg):
        return self.do_quit(arg)


def _kv():
    from ray_amd.experimental import internal_kv

    return internal_kv


def _register(info: dict) -> str | None:
    try:
        kv = _kv()
        if not kv._internal_kv_initialized():
            return None
        key = _PREFIX + uuid.uuid4().hex
        kv._internal_kv_put(key, json.dumps(info), namespace=_NS)
        return key
    except Exception:
        return None


def _unregister(key):
    if key is None:
        return
    try:
        _kv()._internal_kv_del(key, namespace=_NS)
    except Exception:
        pass


def list_breakpoints() -> list:
    kv = _kv()
    out = []
    for k in kv._internal_kv_list(_PREFIX, namespace=_NS) or []:
        k = k.decode() if isinstance(k, bytes) else k
        v = kv._internal_kv_get(k, namespace=_NS)
        if v is not None:
            d = json.loads(v)
            d["key"] = k
            out.append(d)
    return sorted(out, key=lambda d: d.get("created", 0))


def _session(frame, post_mortem_tb=None) -> None:
    from ray_amd import util

    host = util.get_node_ip_address()
    info = {"host": host, "pid": os.getpid(), "created": __import__("time").time()}
    try:
        import ray_amd

        ctx = ray_amd.get_runtime_context()
        info["task_id"] = ctx.get_task_id()
        info["actor_id"] = ctx.get_actor_id()
    except Exception:
        pass
    dbg = RemotePdb(host=host)
    info["port"] = dbg.port
    dbg.key = _register(info)
    dbg.listen()
    if post_mortem_tb is not None:
        dbg.reset()
        dbg.interaction(None, post_mortem_tb)
        dbg._detach()
    else:
        dbg.set_trace(frame)


def set_trace(breakpoint_uuid=None):
    """Break into a debugger in this task/actor (remote) or the driver (local pdb)."""
    from ray_amd._private import worker as _w

    frame = sys._getframe().f_back
    if _w.global_worker.connected and _w.global_worker.mode == _w.WORKER_MODE:
        _session(frame)
    else:
        pdb.Pdb().set_trace(frame)


def post_mortem():
    """Debug the exception currently being handled, remotely when inside a worker."""
    tb = sys.exc_info()[2]
    if tb is None:
        raise ValueError("post_mortem() needs an exception being handled")
    _session(None, post_mortem_tb=tb)


def connect_pdb_client(host: str, port: int, stdin=None, stdout=None):
    """Bridge a terminal to a RemotePdb session until it detaches."""
    import select

    stdin = stdin or sys.stdin
    stdout = stdout or sys.stdout
    s = socket.create_connection((host, port))
    try:
        while True:
            r, _, _ = select.select([s, stdin], [], [])
            if s in r:
                data = s.recv(65536)
                if not data:
                    return
                stdout.write(data.decode(errors="replace").replace("\r\n", "\n"))
                stdout.flush()
            if stdin in r:
                line = stdin.readline()
                if not line:
                    return
                s.sendall(line.encode())
    finally:
        s.close()
