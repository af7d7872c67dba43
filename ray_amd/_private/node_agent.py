"""Worker-node raylet agent (reference: src/ray/raylet/node_manager.cc running on a
non-head node, src/ray/object_manager/object_manager.cc for Pull/Push).

The head raylet (``raylet.py``) is the cluster's scheduler and GCS: it owns every
lease, the actor table and placement groups, and it places work on any registered
node through the native multi-node ``Scheduler``. A worker node runs this agent,
which

  * hosts the node's shared-memory object store (its own ``/dev/shm`` arena and
    spill directory), so workers on the node put/get without IPC;
  * forks worker processes on request from the head (``spawn_worker``) — the workers
    then register with the head directly and are leased like head-node workers;
  * serves object copies to other nodes (``fetch_object``: the reader writes a
    secondary, evictable copy into its own node's store) and frees primaries on the
    owner's request (``free_objects``);
  * dies with its head connection and takes its workers with it, which is how the
    head observes a node failure — unless the head persists its tables
    (RAY_AMD_GCS_STORAGE_PATH): then a lost head is taken to be restarting, and the agent
    keeps its store and workers and re-registers with the new head on the same socket
    (reference: raylet NodeManager::HandleNotifyGCSRestart), giving up after
    RAY_AMD_HEAD_RECONNECT_S (default 30 s). Its actor workers re-attach themselves.
"""

from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time
import traceback

from ray_amd._private.object_store import start_prefault, table_capacity
from ray_amd._native import _core

from . import protocol as P
from . import shm_segment
from .raylet import free_object, node_resources, read_object_bytes, read_object_chunk

_dumps = P.dumps


class NodeAgent:
    def __init__(self, args):
        self.session_dir = args.session_dir
        sock_dir = os.path.join(self.session_dir, "sockets")
        os.makedirs(sock_dir, exist_ok=True)
        self.node_id = _core.random_id(16)
        self.node_hex = self.node_id.hex()
        self.node_ip = "127.0.0.1"
        self.addr = os.path.join(sock_dir, f"raylet_{self.node_hex[:16]}.sock")
        self.store_path, self._store_fd = shm_segment.create(args.store_path)
        self.spill_dir = os.path.join(self.session_dir, f"spill_{self.node_hex[:16]}")
        os.makedirs(self.spill_dir, exist_ok=True)
        self.store = _core.ShmStore(self.store_path, args.object_store_memory, True,
                                    table_capacity(args.object_store_memory))
        start_prefault(self.store, args.object_store_memory)
        from ray_amd._private.object_store import SpillManager

        self.spiller = SpillManager(self.store, self.spill_dir).start()
        self.io = _core.IOLoop()
        self.io.listen_unix(self.addr)
        self.total, self.num_cpus = node_resources(args, self.node_ip, head=False)
        self.labels = json.loads(args.labels or "{}")
        self.procs: dict[int, subprocess.Popen] = {}
        self.stop = False
        self.head_address = args.head_address
        self.head_conn = self.io.connect_unix(args.head_address, 30000)
        if self.head_conn < 0:
            raise ConnectionError(f"cannot reach head raylet at {args.head_address}")
        self.registered = False
        self._register()
        self.reconnect_s = float(os.environ.get("RAY_AMD_HEAD_RECONNECT_S", "30")) \
            if os.environ.get("RAY_AMD_GCS_STORAGE_PATH") else 0.0
        self._head_lost_at = None
        from ray_amd._private.reporter import NodeReporter

        self.reporter = NodeReporter(self.node_hex, self.session_dir).start()
        self._last_report = 0.0

    def _register(self):
        self.io.send(self.head_conn, _dumps((P.HELLO, self.addr, self.node_id)))
        self.io.send(self.head_conn, _dumps((P.REQ, 1, "register_node", (
            self.node_hex, self.total, self.labels, self.addr, self.store_path,
            self.spill_dir, os.getpid(), self.num_cpus))))

    def _try_reconnect(self, now):
        """Head lost with GCS persistence on: retry its socket until the deadline."""
        if now - self._head_lost_at > self.reconnect_s:
            print(f"[ray_amd] node {self.node_hex[:12]}: head did not come back in "
                  f"{self.reconnect_s:.0f}s; exiting", file=sys.stderr, flush=True)
            self.stop = True
            return
        c = self.io.connect_unix(self.head_address, 200)
        if c < 0:
            return
        self.head_conn = c
        self.registered = False
        self._head_lost_at = None
        self._register()
        print(f"[ray_amd] node {self.node_hex[:12]}: re-registered with the restarted head",
              file=sys.stderr, flush=True)

    def reply(self, conn, rid, ok, value):
        if rid:
            self.io.send(conn, _dumps((P.RESP, rid, ok, value)))

    def run(self):
        last = 0.0
        while not self.stop:
            for typ, conn, payload in self.io.poll(50, 1024):
                try:
                    if typ == 0:
                        msg = P.loads(payload)
                        if msg[0] == P.REQ:
                            _, rid, method, args = msg
                            h = getattr(self, "rpc_" + method, None)
                            if h is None:
                                self.reply(conn, rid, False, f"unknown agent method {method}")
                            else:
                                h(conn, rid, *args)
                        elif msg[0] == P.RESP and msg[1] == 1:
                            self.registered = bool(msg[2])
                    elif typ == 2 and conn == self.head_conn:
                        if self.reconnect_s > 0:
                            self.head_conn = None
                            self.registered = False
                            self._head_lost_at = time.monotonic()
                        else:
                            self.stop = True
                except Exception:
                    traceback.print_exc()
            now = time.monotonic()
            if self.head_conn is None and not self.stop:
                self._try_reconnect(now)
                continue
            if self.registered and now - self._last_report >= self.reporter.interval_s:
                self._last_report = now
                sample = self.reporter.latest()
                if sample is not None:  # rid 0: no reply wanted
                    self.io.send(self.head_conn, _dumps((P.REQ, 0, "report_node_stats",
                                                         (self.node_hex, sample))))
            if now - last > 0.5:
                last = now
                for pid, p in list(self.procs.items()):
                    if p.poll() is not None:
                        self.procs.pop(pid, None)
        self.shutdown()

    # ------------------------------------------------------------------ head requests
    def rpc_spawn_worker(self, conn, rid, token, cmd, env, cwd):
        env = dict(env)
        env["RAY_AMD_NODE_ID"] = self.node_hex
        try:
            p = subprocess.Popen(cmd, env=env, cwd=cwd, close_fds=True,
                                 stdout=subprocess.PIPE, stderr=subprocess.PIPE)
            self.procs[p.pid] = p
            self._tee_logs(token, p)
            self.reply(conn, rid, True, p.pid)
        except Exception as e:  # noqa: BLE001
            print(f"[ray_amd] node {self.node_hex[:12]}: worker spawn failed: {e}",
                  file=sys.stderr, flush=True)
            self.reply(conn, rid, False, str(e))

    def _tee_logs(self, token, p):
        """worker-<token>-<pid>.out/.err under <session>/logs, forwarded to this agent's
        stdout / stderr, through one selector thread for the node (as the head raylet)."""
        pump = getattr(self, "_log_pump", None)
        if pump is None:
            from ray_amd._private.log_dedup import LogDeduplicator
            from ray_amd._private.log_pump import LogPump

            pump = self._log_pump = LogPump(LogDeduplicator.from_env())
        d = os.path.join(self.session_dir, "logs")
        os.makedirs(d, exist_ok=True)
        to_driver = os.environ.get("RAY_AMD_LOG_TO_DRIVER", "1") != "0"
        for pipe, ext, out in ((p.stdout, "out", sys.stdout), (p.stderr, "err", sys.stderr)):
            pump.add(pipe, os.path.join(d, f"worker-{token}-{p.pid}.{ext}"),
                     out if to_driver else None, p.pid)

    def rpc_kill_worker(self, conn, rid, pid, graceful):
        p = self.procs.get(pid)
        try:
            if p is not None:
                if not graceful:
                    p.kill()
            else:
                os.kill(pid, signal.SIGKILL)
        except OSError:
            pass
        self.reply(conn, rid, True, None)

    def rpc_fetch_object(self, conn, rid, oid):
        self.reply(conn, rid, True, read_object_bytes(self.store, self.spill_dir, oid))

    def rpc_fetch_object_chunk(self, conn, rid, oid, off, n):
        self.reply(conn, rid, True, read_object_chunk(self.store, self.spill_dir, oid, off, n))

    def rpc_free_objects(self, conn, rid, oids):
        for oid in oids:
            free_object(self.store, self.spill_dir, oid)
        self.reply(conn, rid, True, None)

    def rpc_release_pins_of(self, conn, rid, pid):
        """A worker of this node died: drop its object-store pins, abort its unsealed
        creates (reference: plasma client disconnect -> release all of its objects)."""
        self.reply(conn, rid, True, self.store.release_all_pins_of(int(pid)))

    def rpc_store_stats(self, conn, rid):
        self.reply(conn, rid, True, {"used": self.store.used(-1),
                                     "capacity": self.store.capacity(-1),
                                     "num_objects": self.store.num_objects()})

    def rpc_ping(self, conn, rid):
        self.reply(conn, rid, True, self.node_hex)

    def rpc_shutdown(self, conn, rid):
        self.reply(conn, rid, True, None)
        self.stop = True

    def shutdown(self):
        for p in list(self.procs.values()):
            try:
                p.kill()
            except OSError:
                pass
        for p in list(self.procs.values()):
            try:
                p.wait(timeout=2)
            except Exception:
                pass
        self.spiller.stop()
        shm_segment.release(self.store_path, self._store_fd)
        self.io.stop()
