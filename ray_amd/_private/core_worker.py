"""CoreWorker: the per-process runtime (reference: src/ray/core_worker/core_worker.cc,
reference_count.cc, task_manager.cc, transport/normal_task_submitter.cc,
transport/actor_task_submitter.cc, task_receiver.cc).

Threads:
  * native IOLoop thread (C++): socket I/O, frame parsing, GIL-free.
  * dispatcher thread: pulls frames, runs protocol handlers (never blocks).
  * main thread: user code; in worker processes also the task executor loop.
  * actor pools: thread pool (max_concurrency>1 / concurrency groups) or an
    asyncio loop thread (async actors).

Ownership: the process that creates an ObjectRef (by .remote() or put) owns it.
Owners keep value (inline bytes for small objects, or the shm store entry),
readiness, borrower set and containment pins. Borrowers register with the owner
(async when ordering is implied by the channel, synchronously otherwise — see
``_register_borrow``) and deregister when their local count reaches zero.
"""

from __future__ import annotations

import collections
import ctypes
import hashlib
import os
import queue
import sys
import threading
import time
import traceback

import cloudpickle

from ray_amd._native import _core
from ray_amd.util.tracing import tracing_helper as _tracing
from ray_amd.exceptions import (ObjectReconstructionFailedError,
                                ObjectReconstructionFailedLineageEvictedError,
                                ObjectReconstructionFailedMaxAttemptsExceededError)
from ray_amd.exceptions import OutOfMemoryError
from ray_amd.exceptions import (GetTimeoutError, ObjectLostError, OwnerDiedError,
                                RayActorError, RayTaskError, TaskCancelledError,
                                WorkerCrashedError, ActorDiedError)

from . import protocol as P
from . import serialization as ser
from .ids import object_id_for_put, object_id_for_return

INLINE_MAX = 100 * 1024  # reference: max_direct_call_object_size
ARGS_INLINE_MAX = 100 * 1024
LEASE_IDLE_S = 0.02
# Lease requests in flight per scheduling class. The reference caps this at the number of
# nodes (ray_config_def.h max_pending_lease_requests_per_scheduling_category = -1 ->
# #nodes) and requests more as grants return; 64 here flooded the raylet with requests it
# rescanned on every scheduling pass: with 4, multi-client async tasks went from 5.6-8.8k
# to 13-21.5k tasks/s on the 8-CPU node (profiles/microbenchmark_r5.md).
MAX_PENDING_LEASES_PER_KEY = int(os.environ.get("RAY_AMD_MAX_PENDING_LEASES", "4"))
# Tasks in flight per leased worker while the node is saturated for the task's scheduling
# class (lease requests unanswered for PIPELINE_AFTER_S): the next task waits in the
# worker's queue instead of a full owner -> worker round trip after each reply. A worker
# whose running task blocks in get/wait hands its queued tasks back, and an owner whose
# lease goes idle steals a queued task back from a busy one (work stealing), so a pipelined
# task never waits behind a task that depends on it. RAY_AMD_PIPELINE_DEPTH=1 disables it.


def _drain(q: collections.deque) -> list:
    """Pop everything from a deque that other threads also pop from (a threaded actor's
    pool threads send replies concurrently): popleft until empty, never a length taken
    before the pops."""
    out = []
    try:
        while True:
            out.append(q.popleft())
    except IndexError:
        pass
    return out

PIPELINE_DEPTH = max(1, int(os.environ.get("RAY_AMD_PIPELINE_DEPTH", "2")))
PIPELINE_AFTER_S = float(os.environ.get("RAY_AMD_PIPELINE_AFTER_MS", "5")) / 1000.0

_dumps = P.dumps
_loads = P.loads


class _Owned:
    __slots__ = ("ready", "inline", "in_store", "callbacks", "borrowers", "contained",
                 "release_when_ready", "task_id", "size", "node", "recon", "lineage_refs",
                 "accessed")

    def __init__(self, task_id=None):
        self.accessed = False  # value read (get / await / passed as an argument)
        self.ready = False
        self.inline = None
        self.in_store = False
        self.callbacks = None
        self.borrowers = None
        self.contained = None
        self.release_when_ready = False
        self.task_id = task_id
        self.size = 0
        self.node = None
        self.recon = 0  # times this object was reconstructed from lineage
        # lineage entries (finished task specs) that list this object as an argument: the
        # VALUE is freed with the last in-scope ref, but this metadata is kept so the
        # object can be re-created if a dependent's reconstruction needs it
        self.lineage_refs = 0


# Lineage (creating-task specs of stored task returns) kept per owner. A lineage entry
# holds only argument ids, never argument values (reference: reference_count.cc lineage
# ref counts). The oldest entries are dropped beyond either bound (their objects then
# fail with LineageEvicted if lost); reference default max_lineage_bytes = 1 GiB.
LINEAGE_MAX = 20000
LINEAGE_MAX_BYTES = 1 << 30


class _CopyLost(Exception):
    """Internal: the stored copy of a ready object could not be read."""

    def __init__(self, node):
        self.node = node


class _Remote:
    """Borrower-side view of an object owned elsewhere."""

    __slots__ = ("state", "inline", "error", "callbacks", "node")

    def __init__(self):
        self.state = 0  # 0 unknown, 1 requested, 2 ready, 3 failed
        self.inline = None
        self.error = None
        self.callbacks = []
        self.node = None  # node holding the primary copy (hex), None = ours


class _Lease:
    __slots__ = ("addr", "lease_id", "inflight", "idle_since", "key", "gpu_ids", "worker_id")

    def __init__(self, addr, lease_id, key, gpu_ids, worker_id):
        self.addr = addr
        self.lease_id = lease_id
        self.inflight = {}
        self.idle_since = time.monotonic()
        self.key = key
        self.gpu_ids = gpu_ids
        self.worker_id = worker_id


class _ActorConn:
    __slots__ = ("actor_id", "state", "addr", "queue", "inflight", "seq", "subscribed",
                 "death", "max_task_retries", "num_restarts", "lost", "release_when_idle")

    def __init__(self, actor_id):
        self.actor_id = actor_id
        # every handle is gone but submitted calls are still queued / running: the actor
        # is released once they have replied (reference: out-of-scope actors finish the
        # tasks already submitted to them)
        self.release_when_idle = False
        self.state = P.PENDING_CREATION
        self.addr = None
        self.queue = collections.deque()
        self.inflight = {}
        self.seq = 0
        self.subscribed = False
        self.death = None
        self.max_task_retries = 0
        self.num_restarts = 0
        # non-retriable in-flight tasks of a lost connection, failed once the actor's
        # death cause arrives (e.g. the memory monitor killed it) or after a grace period
        self.lost = []


class _Stream:
    __slots__ = ("items", "done", "error_ref", "cv_waiters", "total", "conn", "consumed", "bp")

    def __init__(self, bp=0):
        self.items = {}
        self.done = False
        self.error_ref = None
        self.total = None
        self.conn = None  # the executing worker's connection (backpressure acks)
        self.consumed = 0
        self.bp = bp  # _generator_backpressure_num_objects (0: unbounded)


class _Waiter:
    __slots__ = ("need", "done", "ev")

    def __init__(self, need):
        self.need = need
        self.done = set()
        self.ev = threading.Event()

    def hit(self, oid):
        self.done.add(oid)
        if len(self.done) >= self.need:
            self.ev.set()


def _raise_in_thread(tid: int, exc_type) -> None:
    ctypes.pythonapi.PyThreadState_SetAsyncExc(ctypes.c_ulong(tid), ctypes.py_object(exc_type))


class CoreWorker:
    def __init__(self, *, mode: str, session_dir: str, raylet_addr: str, worker_id: bytes,
                 job_id: int | None = None, namespace: str | None = None,
                 gpu_ids=None, node_id=None, startup_token=None, runtime_env=None):
        self.mode = mode  # "driver" | "worker"
        self.session_dir = session_dir
        self.worker_id = worker_id
        self.addr = os.path.join(session_dir, "sockets", worker_id.hex()[:24] + ".sock")
        self.io = _core.IOLoop()
        self.io.listen_unix(self.addr)
        self.lock = threading.RLock()
        self._ready_cv = threading.Condition(self.lock)
        self._wake_targets: list = []  # ready-seq values at which a waiter wants a wake-up
        self._ready_log = collections.deque(maxlen=1 << 16)
        self._ready_owned: set = set()  # owned oids that are ready (set algebra in wait)
        self._ready_seq = 0
        self.raylet_addr = raylet_addr
        self.conns: dict[str, int] = {}
        self.conn_addr: dict[int, str] = {}
        self._rid = 1
        self._rpc_cb: dict[int, object] = {}
        # ownership
        self.refs: dict[bytes, list] = {}  # oid -> [count, owner, registered]
        self.owned: dict[bytes, _Owned] = {}
        self.remote: dict[bytes, _Remote] = {}
        self.streams: dict[bytes, _Stream] = {}
        # submission
        self.sched_queues: dict = collections.defaultdict(collections.deque)
        self.leases: dict = collections.defaultdict(list)
        self.pending_leases: dict = collections.defaultdict(int)
        self._lease_wait_t: dict = {}  # key -> when its lease requests last went unanswered
        self._stealing: set = set()  # tids with a STEAL in flight
        self.pipeline_stats = collections.Counter()  # pipelined / requeued / steals
        self.task_specs: dict[bytes, dict] = {}  # tid -> spec (pending/running)
        # tid -> spec of FINISHED normal tasks whose stored returns are still owned: the
        # lineage re-executed when a primary copy is lost (object_recovery_manager.cc)
        self.lineage: "collections.OrderedDict[bytes, dict]" = collections.OrderedDict()
        self.lineage_bytes = 0
        self.lineage_evicted: set = set()
        # oid -> metadata of freed objects still named as arguments by lineage entries
        self.lineage_objs: dict[bytes, _Owned] = {}
        self.task_lease: dict[bytes, _Lease] = {}
        self.actors: dict[bytes, _ActorConn] = {}
        self.actor_handle_counts: collections.Counter = collections.Counter()
        self.actor_escaped: set = set()
        self.exported: set = set()
        self.fn_cache: dict = {}
        self.put_index = 0
        self.task_counter = 0
        # execution (worker side)
        self.exec_queue: queue.Queue = queue.Queue()
        self.current_task = threading.local()
        self.running: dict[bytes, int] = {}  # tid -> thread ident
        self.cancelled: set = set()
        # cancellation: tasks submitted while executing task P (recursive cancel), the
        # asyncio tasks of an async actor, and whether the main thread is inside user code
        # (SIGINT is honoured only there: never while arguments are being deserialised)
        self._children: dict[bytes, list] = {}
        self._async_tasks: dict = {}
        self._main_interruptible = False
        self._sigint_installed = False
        self.actor_instance = None
        self.actor_id = None
        self.actor_spec = None
        self.actor_pools: dict = {}
        self.async_loop = None
        self.exiting = False
        self.blocked_depth = 0
        self.task_events = collections.deque()  # append/popleft are atomic across threads
        self._events_flushed = 0.0
        self.gpu_ids = gpu_ids or []
        self.node_id = node_id
        self._ns = namespace
        self.job_id = job_id
        self.local_mode = False
        self.runtime_env = runtime_env or {}
        self.store = None
        # connect to raylet
        self.raylet_conn = self._connect(raylet_addr)
        self._stopped = False
        self.dispatcher = threading.Thread(target=self._dispatch_loop, name="ray_amd-dispatch",
                                           daemon=True)
        self.dispatcher.start()
        reg = self.call_raylet("register", mode, worker_id, os.getpid(), self.addr, job_id,
                               namespace, startup_token, os.environ.get("RAY_AMD_NODE_ID"))
        from .object_store import ObjectStore

        self.node_id = reg["node_id"]
        self.job_id = reg["job_id"]
        self._ns = reg.get("namespace") or namespace
        self.node_ip = reg.get("node_ip", "127.0.0.1")
        self.store = ObjectStore(reg["store_path"], reg["spill_dir"], create=False)
        self.cluster_info = reg
        self.node_hex = self.node_id.hex()
        self._node_addrs: dict[str, str] = {}
        self.task_id_base = os.urandom(12)

    @property
    def namespace(self):
        """The namespace of the task running on this thread (its driver's), else this
        process's own."""
        return getattr(self.current_task, "ns", None) or self._ns

    @namespace.setter
    def namespace(self, v):
        self._ns = v

    # ------------------------------------------------------------------ connections
    def _connect(self, addr: str) -> int:
        c = self.io.connect_unix(addr, 30000)
        if c < 0:
            raise ConnectionError(f"cannot connect to {addr}")
        self.conns[addr] = c
        self.conn_addr[c] = addr
        self.io.send(c, _dumps((P.HELLO, self.addr, self.worker_id)))
        return c

    def _conn(self, addr: str) -> int:
        c = self.conns.get(addr)
        if c is not None:
            return c
        with self.lock:
            c = self.conns.get(addr)
            if c is not None:
                return c
            return self._connect(addr)

    def send(self, addr: str, msg) -> bool:
        try:
            c = self._conn(addr)
        except ConnectionError:
            return False
        ok = self.io.send(c, _dumps(msg))
        return ok

    def _next_rid(self) -> int:
        with self.lock:
            self._rid += 1
            return self._rid

    def call_async(self, addr: str, method: str, args: tuple, cb) -> None:
        """cb(ok, value) runs on the dispatcher thread."""
        rid = self._next_rid()
        self._rpc_cb[rid] = (cb, addr)
        if not self.send(addr, (P.REQ, rid, method, args)):
            self._rpc_cb.pop(rid, None)
            cb(False, ConnectionError(f"peer {addr} unreachable"))

    def call(self, addr: str, method: str, *args, timeout: float | None = None):
        if threading.current_thread() is self.dispatcher:
            raise RuntimeError("blocking RPC from the dispatcher thread")
        box = []
        ev = threading.Event()

        def cb(ok, value):
            box.append((ok, value))
            ev.set()

        self.call_async(addr, method, args, cb)
        if not ev.wait(timeout):
            raise GetTimeoutError(f"RPC {method} to {addr} timed out")
        ok, value = box[0]
        if not ok:
            if isinstance(value, BaseException):
                raise value
            raise RuntimeError(value)
        return value

    def call_raylet(self, method: str, *args, timeout: float | None = None):
        return self.call(self.raylet_addr, method, *args, timeout=timeout)

    def notify_raylet(self, method: str, *args):
        self.send(self.raylet_addr, (P.REQ, 0, method, args))

    # ------------------------------------------------------------------ dispatcher
    def _dispatch_loop(self):
        io = self.io
        handlers = {
            P.REQ: self._on_req,
            P.RESP: self._on_resp,
            P.PUSH: self._on_push,
            P.HELLO: self._on_hello,
            P.TASK: self._on_task,
            P.TASK_REPLY: self._on_task_reply,
            P.STREAM_ITEM: self._on_stream_item,
            P.STREAM_ACK: self._on_stream_ack,
            P.STEAL: self._on_steal,
        }
        # poll timeout: messages wake the loop at once; the timeout only paces the periodic
        # work below (lease reaping, task-event flushes). Every wake takes the GIL from the
        # process's compute thread (a Train worker's launch loop), so it is configurable.
        poll_ms = int(os.environ.get("RAY_AMD_POLL_MS", "10"))
        prof_dir = os.environ.get("RAY_AMD_WORKER_CPROFILE")  # diagnostics (worker_main.py)
        prof, prof_t = None, 0.0
        if prof_dir:
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        while not self._stopped:
            if prof is not None and time.monotonic() - prof_t > 2.0:
                prof_t = time.monotonic()
                prof.disable()
                prof.dump_stats(os.path.join(prof_dir,
                                             f"{self.mode}-{os.getpid()}-dispatch.prof"))
                prof.enable()
            try:
                events = io.poll(poll_ms, 4096)
            except Exception:
                break
            for typ, conn, payload in events:
                try:
                    if typ == 0:
                        msg = _loads(payload)
                        h = handlers.get(msg[0])
                        if h is not None:
                            h(conn, msg)
                    elif typ == 2:
                        self._on_conn_closed(conn)
                except Exception:
                    if not self._stopped:
                        traceback.print_exc()
            try:
                self._reap_idle_leases()
                # workers flush every 0.1 s (their task events mostly travel on the task
                # replies), drivers every 0.5 s; state queries flush the caller first
                if self.task_events and (
                        len(self.task_events) > 4096 or time.monotonic() - self._events_flushed
                        > (0.1 if self.mode == "worker" else 0.5)):
                    self._flush_task_events()
            except Exception:
                if not self._stopped:
                    traceback.print_exc()

    def _on_hello(self, conn, msg):
        addr = msg[1]
        self.conn_addr[conn] = addr
        with self.lock:
            if addr not in self.conns:
                self.conns[addr] = conn

    def _on_resp(self, conn, msg):
        _, rid, ok, value = msg
        ent = self._rpc_cb.pop(rid, None)
        if ent is not None:
            ent[0](ok, value)

    def _reply(self, conn, rid, ok, value):
        if rid:
            addr = self.conn_addr.get(conn)
            if addr is not None and addr in self.conns:
                self.send(addr, (P.RESP, rid, ok, value))
            else:
                self.io.send(conn, _dumps((P.RESP, rid, ok, value)))

    def _on_req(self, conn, msg):
        _, rid, method, args = msg
        h = getattr(self, "_rpc_" + method, None)
        if h is None:
            self._reply(conn, rid, False, f"unknown method {method}")
            return
        try:
            h(conn, rid, *args)
        except Exception as e:  # noqa: BLE001
            traceback.print_exc()
            self._reply(conn, rid, False, repr(e))

    def _on_conn_closed(self, conn):
        addr = self.conn_addr.pop(conn, None)
        if addr is None:
            return
        with self.lock:
            if self.conns.get(addr) == conn:
                del self.conns[addr]
        if addr == self.raylet_addr:
            if not self._stopped and self.mode == "worker":
                if getattr(self, "_reattaching", False):
                    return  # the re-attach loop sees its call fail and reconnects
                if self._can_reattach():
                    self._reattaching = True
                    threading.Thread(target=self._reattach_loop, name="ray_amd-reattach",
                                     daemon=True).start()
                    return
                os._exit(1)
            return
        # fail outstanding RPCs to that peer
        for rid, (cb, a) in list(self._rpc_cb.items()):
            if a == addr:
                self._rpc_cb.pop(rid, None)
                cb(False, ConnectionError(f"peer {addr} died"))
        # borrowers that died
        with self.lock:
            for o in self.owned.values():
                if o.borrowers and addr in o.borrowers:
                    del o.borrowers[addr]
        dead = [oid for oid, o in list(self.owned.items())]
        for oid in dead:
            self._maybe_free(oid)
        # leased worker died -> fail/retry its tasks
        self._on_worker_lost(addr)
        # actor died -> handled through raylet PUSH, but fail in-flight fast
        for ac in list(self.actors.values()):
            if ac.addr == addr and ac.state == P.ALIVE:
                self._on_actor_conn_lost(ac)

    def _can_reattach(self) -> bool:
        """An actor worker on a node other than the head's outlives a head restart when the
        head persists its tables (the restarted head awaits re-attachment)."""
        return (self.actor_id is not None and bool(os.environ.get("RAY_AMD_GCS_STORAGE_PATH"))
                and self.node_hex != (self.cluster_info or {}).get("head_node_id"))

    def _reattach_loop(self):
        """Reconnect to the restarted head on its socket, register again and re-attach this
        actor (reference: core_worker.cc re-subscribing after a GCS restart). Gives up —
        the process exits as before — after RAY_AMD_HEAD_RECONNECT_S or when the head has
        re-created or dropped the actor."""
        deadline = time.monotonic() + float(os.environ.get("RAY_AMD_HEAD_RECONNECT_S", "30"))
        while time.monotonic() < deadline and not self._stopped:
            c = self.io.connect_unix(self.raylet_addr, 200)
            if c < 0:
                continue
            with self.lock:
                self.conns[self.raylet_addr] = c
                self.conn_addr[c] = self.raylet_addr
            self.io.send(c, _dumps((P.HELLO, self.addr, self.worker_id)))
            while time.monotonic() < deadline:
                try:
                    self.call_raylet("register", "worker", self.worker_id, os.getpid(),
                                     self.addr, self.job_id, self._ns, None, self.node_hex,
                                     timeout=5)
                    ok = self.call_raylet("reattach_actor", self.actor_id, timeout=5)
                except Exception:  # noqa: BLE001 - the head went away again: reconnect
                    break
                if ok is True:
                    self._reattaching = False
                    return
                if ok != "retry":
                    os._exit(1)
                time.sleep(0.2)
        os._exit(1)

    def _on_push(self, conn, msg):
        _, topic, data = msg
        if topic == "actor":
            self._on_actor_update(*data)
        elif topic == "exit":
            self.exiting = True
            os._exit(0)

    # ------------------------------------------------------------------ references
    # A borrowed id's entry in self.refs is [local count, owner, credits]: credits = how
    # many borrower registrations the owner holds for this process (one per hand-over
    # the owner pinned for us — a reply's contained refs — plus our own add_borrower).
    # The owner counts registrations per borrower and the release message returns all
    # credits at once, so a release racing a fresh hand-over of the same id (a prefetched
    # reply already on its way) cannot drop the owner's count to zero early.
    def add_local_ref(self, oid: bytes, owner: str, deserialized: bool = False):
        register = False
        with self.lock:
            e = self.refs.get(oid)
            if e is None:
                e = self.refs[oid] = [1, owner, 0]
                if owner != self.addr and owner:
                    e[2] = 1
                    register = True
            else:
                e[0] += 1
        if register:
            self._register_borrow(oid, owner)

    def _add_borrow_credit(self, oid: bytes, owner: str):
        """The sender of a reply pinned `oid` at its owner for us: one credit, and no
        add_borrower of our own for the pins about to be made."""
        if not owner or owner == self.addr:
            return
        with self.lock:
            e = self.refs.get(oid)
            if e is None:
                self.refs[oid] = [0, owner, 1]
            else:
                e[2] += 1

    def _register_borrow(self, oid, owner):
        ctx = ser.current_deser_context()
        anchor = ctx.anchor if ctx is not None else None
        if anchor is None or anchor == owner or threading.current_thread() is self.dispatcher:
            self.send(owner, (P.REQ, 0, "add_borrower", (oid, self.addr)))
        else:
            try:
                self.call(owner, "add_borrower", oid, self.addr, timeout=30)
            except Exception:
                pass

    def remove_local_ref(self, oid: bytes):
        notify = None
        with self.lock:
            e = self.refs.get(oid)
            if e is None:
                return
            e[0] -= 1
            if e[0] > 0:
                return
            del self.refs[oid]
            owned = e[1] == self.addr
            if not owned:
                self.remote.pop(oid, None)
                if e[2]:
                    notify = e[1]
        if owned:
            self._maybe_free(oid)
        elif notify and not self._stopped:
            self.send(notify, (P.REQ, 0, "remove_borrower", (oid, self.addr, e[2])))

    def _maybe_free(self, oid: bytes):
        contained = None
        with self.lock:
            o = self.owned.get(oid)
            if o is None or oid in self.refs or o.borrowers:
                return
            if not o.ready:
                o.release_when_ready = True
                return
            del self.owned[oid]
            self._ready_owned.discard(oid)
            unhandled = o.inline if (o.inline is not None and not o.accessed) else None
            contained = o.contained
            o.contained = None
            in_store = o.in_store
            node = o.node
            tid = o.task_id
            if o.lineage_refs > 0 and tid is not None and tid in self.lineage:
                # a dependent's lineage names it: keep the metadata, free the value
                o.ready = False
                o.inline = None
                o.in_store = False
                o.node = None
                self.lineage_objs[oid] = o
            else:
                self._drop_lineage_if_unused(tid)
        if in_store:
            self._delete_stored(oid, node)
        del contained
        if unhandled is not None:
            self._report_unhandled(unhandled)

    def _report_unhandled(self, inline):
        """An error object freed without ever being read (reference: core_worker memory
        store unhandled-exception handler -> "Unhandled error" on stderr)."""
        if "RAY_IGNORE_UNHANDLED_ERRORS" in os.environ or self._stopped:
            return
        try:
            if ser.header(memoryview(inline))[0] != ser.KIND_ERROR:
                return
            _, err = ser.deserialize(inline)
        except Exception:  # noqa: BLE001
            return
        # only task failures, as the reference (memory_store.cc IsUnhandledError:
        # TASK_EXECUTION_EXCEPTION / WORKER_DIED; an actor that died or was killed is not)
        from ray_amd.exceptions import WorkerCrashedError

        if isinstance(err, RayActorError) or not isinstance(err, (RayTaskError,
                                                                   WorkerCrashedError)):
            return
        try:
            sys.stderr.write("Unhandled error (suppress with "
                             f"'RAY_IGNORE_UNHANDLED_ERRORS=1'): {err}\n")
            sys.stderr.flush()
        except Exception:  # noqa: BLE001
            pass

    def _lineage_in_use(self, tid) -> bool:
        spec = self.lineage.get(tid)
        if spec is None:
            return False
        for i in range(max(spec["nret"], 0)):
            r = object_id_for_return(tid, i + 1)
            if r in self.owned or r in self.lineage_objs:
                return True
        return False

    def _drop_lineage_if_unused(self, tid):
        """(lock held) Delete the lineage entry of `tid` once none of its returns is owned
        or named by another lineage entry; cascades through the argument chain."""
        work = [tid]
        while work:
            t = work.pop()
            if t is None or t not in self.lineage or self._lineage_in_use(t):
                continue
            spec = self.lineage.pop(t)
            work.extend(self._release_lineage_args(spec))

    def _release_lineage_args(self, spec):
        """(lock held) Drop the lineage refs a spec holds on its arguments. Returns the task
        ids whose lineage may have become unused."""
        self.lineage_bytes -= spec.pop("_lbytes", 0)
        out = []
        for a in spec.pop("_largs", ()):
            o = self.owned.get(a)
            if o is None:
                o = self.lineage_objs.get(a)
                if o is None:
                    continue
                o.lineage_refs -= 1
                if o.lineage_refs <= 0:
                    del self.lineage_objs[a]
                    out.append(o.task_id)
            else:
                o.lineage_refs -= 1
        return out

    def _delete_stored(self, oid, node):
        """Free a primary copy: in our node's store, or via its node's agent."""
        if node is None or node == self.node_hex:
            if self.store is None:
                return
            try:
                self.store.delete(oid)
                from . import gpu_object_store

                gpu_object_store.free_sub_objects(self.store.store, oid)
            except Exception:
                pass
            return
        if self._stopped:
            return
        addr = self._node_addrs.get(node)
        if addr is not None:
            self.send(addr, (P.REQ, 0, "free_objects", ([oid],)))
            return

        def got(ok, a, oid=oid, node=node):
            if ok and a:
                self._node_addrs[node] = a
                self.send(a, (P.REQ, 0, "free_objects", ([oid],)))

        self.call_async(self.raylet_addr, "node_addr", (node,), got)

    def _node_addr(self, node):
        a = self._node_addrs.get(node)
        if a is None:
            a = self.call_raylet("node_addr", node, timeout=30)
            if a is not None:
                self._node_addrs[node] = a
        return a

    PULL_CHUNK = 16 << 20  # bytes per pull request
    PULL_PARALLEL = 4  # chunk requests in flight

    def _fetch_remote(self, oid, node):
        """Pull a copy of an object whose primary lives on another node into our node's
        store as an unpinned (evictable) secondary copy (reference: ObjectManager::Pull with
        chunked transfers). The first request returns the size; the remaining chunks are
        requested PULL_PARALLEL at a time and written straight into the local store entry.
        Returns a buffer over the local copy, or None if the node no longer has it."""
        addr = self._node_addr(node)
        if addr is None:
            return None
        C = self.PULL_CHUNK
        try:
            first = self.call(addr, "fetch_object_chunk", oid, 0, C, timeout=120)
        except Exception:
            return None
        if first is None:
            return None
        total, head = first
        if self.store.contains(oid):
            buf = self.store.get_buffer(oid)
            if buf is not None:
                return buf
        try:
            off0 = self.store._alloc(oid, total, False, wait=False)
        except Exception:
            off0 = None
        if off0 is None:  # store full: assemble on the heap and serve this read from it
            data = bytearray(total)
            data[:len(head)] = head
            ok = self._pull_rest(addr, oid, total, len(head),
                                 lambda o, b: data.__setitem__(slice(o, o + len(b)), b))
            return memoryview(bytes(data)) if ok else None
        try:
            self.store.store.write(off0, head)
            ok = self._pull_rest(addr, oid, total, len(head),
                                 lambda o, b: self.store.store.write(off0 + o, b))
        except BaseException:
            self.store.store.abort(oid)
            raise
        if not ok:
            self.store.store.abort(oid)
            return None
        self.store.store.seal(oid)
        return self.store.get_buffer(oid)

    def _pull_rest(self, addr, oid, total, start, sink) -> bool:
        import concurrent.futures as cf

        C = self.PULL_CHUNK
        offs = list(range(start, total, C))
        if not offs:
            return True

        def one(o):
            r = self.call(addr, "fetch_object_chunk", oid, o, C, timeout=120)
            if r is None:
                raise KeyError(oid)
            sink(o, r[1])

        try:
            with cf.ThreadPoolExecutor(self.PULL_PARALLEL) as ex:
                list(ex.map(one, offs))
        except Exception:
            return False
        return True

    def _rpc_add_borrower(self, conn, rid, oid, addr):
        with self.lock:
            o = self.owned.get(oid)
            if o is not None:
                if o.borrowers is None:
                    o.borrowers = {}
                o.borrowers[addr] = o.borrowers.get(addr, 0) + 1
        self._reply(conn, rid, True, o is not None)

    def _rpc_remove_borrower(self, conn, rid, oid, addr, n=1):
        with self.lock:
            o = self.owned.get(oid)
            if o is not None and o.borrowers and addr in o.borrowers:
                left = o.borrowers[addr] - n
                if left > 0:
                    o.borrowers[addr] = left
                else:
                    del o.borrowers[addr]
        self._maybe_free(oid)
        self._reply(conn, rid, True, None)

    # ------------------------------------------------------------------ object values
    def _mark_ready(self, oid, inline=None, in_store=False, contained=None, size=0, node=None):
        cbs = None
        free = False
        if node == self.node_hex:
            node = None
        with self.lock:
            o = self.owned.get(oid)
            if o is None:
                # released while pending
                if in_store:
                    self._delete_stored(oid, node)
                return
            if o.ready:
                return
            o.inline = inline
            o.in_store = in_store
            o.contained = contained
            o.size = size
            o.node = node
            o.ready = True
            self._ready_owned.add(oid)
            self._ready_log.append(oid)
            self._ready_seq += 1
            # wake waiters only once enough objects became ready to possibly satisfy one:
            # a get() of 1000 refs is woken once, not 1000 times (each wake-up takes the GIL
            # from the dispatcher thread that is delivering the replies)
            wt = self._wake_targets
            if wt and self._ready_seq >= min(wt):
                self._ready_cv.notify_all()
            cbs = o.callbacks
            o.callbacks = None
            free = o.release_when_ready
        if cbs:
            for cb in cbs:
                try:
                    cb(oid)
                except Exception:
                    traceback.print_exc()
        if free:
            self._maybe_free(oid)

    def put_object(self, value, owner_pinned=True) -> "object":
        from ray_amd.object_ref import ObjectRef

        with self.lock:
            self.put_index += 1
            idx = self.put_index
        oid = object_id_for_put(self._current_task_id(), idx)
        sobj = ser.serialize(value, oid)
        return self._store_owned(oid, sobj, ObjectRef)

    def put_serialized_object(self, oid, sobj):
        from ray_amd.object_ref import ObjectRef

        return self._store_owned(oid, sobj, ObjectRef)

    def _store_owned(self, oid, sobj, ObjectRef):
        o = _Owned()
        with self.lock:
            self.owned[oid] = o
        ref = ObjectRef(oid, self.addr, _cw_obj=self)
        contained = sobj.refs or None
        if sobj.total <= INLINE_MAX and not sobj.gpu:
            self._mark_ready(oid, inline=sobj.to_bytes(), contained=contained, size=sobj.total)
        else:
            self.store.put_serialized(oid, sobj, pinned=True)
            self._mark_ready(oid, in_store=True, contained=contained, size=sobj.total)
        return ref

    def _current_task_id(self) -> bytes:
        t = getattr(self.current_task, "tid", None)
        if t is not None:
            return t
        return self.task_id_base + (0).to_bytes(4, "little")

    def _on_ready(self, oid: bytes, cb) -> bool:
        """Register cb(oid) for readiness. Returns True if already ready (cb not called)."""
        with self.lock:
            o = self.owned.get(oid)
            if o is not None:
                if o.ready:
                    return True
                if o.callbacks is None:
                    o.callbacks = []
                o.callbacks.append(cb)
                return False
            e = self.refs.get(oid)
            owner = e[1] if e else None
            r = self.remote.get(oid)
            if r is None:
                r = self.remote[oid] = _Remote()
            if r.state in (2, 3):
                return True
        if owner is None or owner == self.addr:
            # not owned by us and no owner known: treat as lost
            with self.lock:
                r.state = 3
                r.error = ObjectLostError(oid.hex())
            return True
        if self.store is not None and self.store.contains(oid):
            with self.lock:
                r.state = 2
            return True
        with self.lock:
            r.callbacks.append(cb)
            need_req = r.state == 0
            if need_req:
                r.state = 1
        if need_req:
            def on_reply(ok, value, oid=oid):
                cbs = []
                with self.lock:
                    rr = self.remote.get(oid)
                    if rr is None:
                        rr = _Remote()
                    if ok and value[0] == "inline":
                        rr.state, rr.inline = 2, value[1]
                    elif ok and value[0] == "store":
                        rr.state = 2
                        if value[1] is not None and value[1] != self.node_hex:
                            rr.node = value[1]
                    else:
                        rr.state = 3
                        rr.error = (OwnerDiedError(oid.hex()) if not ok else
                                    ObjectLostError(oid.hex()))
                    cbs, rr.callbacks = rr.callbacks, []
                for c in cbs:
                    c(oid)

            self.call_async(owner, "get_object", (oid,), on_reply)
        return False

    def _rpc_get_object(self, conn, rid, oid):
        def respond(_oid=oid):
            with self.lock:
                o = self.owned.get(oid)
                if o is None:
                    val = ("lost", None)
                elif o.inline is not None:
                    val = ("inline", o.inline)
                    o.accessed = True  # a borrower reads it (no false "Unhandled error")
                else:
                    val = ("store", o.node or self.node_hex)
            self._reply(conn, rid, True, val)

        with self.lock:
            o = self.owned.get(oid)
            if o is None:
                self._reply(conn, rid, True, ("lost", None))
                return
            if not o.ready:
                if o.callbacks is None:
                    o.callbacks = []
                o.callbacks.append(lambda _o: respond())
                return
        respond()

    def _value_of(self, oid: bytes, anchor: str | None):
        """Deserialize a READY object. Raises the stored error for error objects. A lost
        stored copy is recovered by re-executing its creating task (lineage)."""
        for _ in range(8):
            try:
                return self._value_of_once(oid, anchor)
            except _CopyLost as lost:
                self._recover(oid, lost.node)
        raise ObjectReconstructionFailedError(oid.hex(), "object kept getting lost")

    def _recover(self, oid, failed_node):
        """Block until a lost object is available again (owner: re-execute lineage;
        borrower: ask the owner to). Raises the reconstruction error if it cannot."""
        with self.lock:
            owned = oid in self.owned
            e = self.refs.get(oid)
            owner = e[1] if e else None
        if owned:
            err = self._reconstruct(oid, failed_node)
            if err is not None:
                raise err
            self.wait_refs([oid], 1, None)
            return
        if owner is None or owner == self.addr:
            raise ObjectLostError(oid.hex())
        try:
            ok, err = self.call(owner, "recover_object", oid, failed_node, timeout=None)
        except Exception:
            raise OwnerDiedError(oid.hex()) from None
        if not ok:
            raise err
        with self.lock:
            self.remote.pop(oid, None)  # stale location: ask the owner again
        self.wait_refs([oid], 1, None)

    def _reconstruct(self, oid, failed_node=None):
        """Owner side: resubmit the task that created `oid`. Returns None when the object
        is (or will become) available, else the error to raise."""
        with self.lock:
            o = self.owned.get(oid)
            revived = False
            if o is None:
                o = self.lineage_objs.get(oid)
                if o is None:
                    return ObjectLostError(oid.hex())
                revived = True  # a freed argument a dependent's re-execution needs
            elif not o.ready:
                return None  # a reconstruction is already running
            elif o.inline is not None or (o.node or None) != (failed_node or None):
                return None  # already recovered (another caller saw the loss first)
            tid = o.task_id
            if tid is None:  # ray.put objects have no lineage (reference semantics)
                return ObjectLostError(oid.hex())
            spec = self.lineage.get(tid)
            if spec is None:
                if tid in self.lineage_evicted:
                    return ObjectReconstructionFailedLineageEvictedError(
                        oid.hex(), "the lineage of the creating task was evicted")
                return ObjectReconstructionFailedError(oid.hex(), "no lineage for the task")
            if spec["retries"] == 0:
                return ObjectReconstructionFailedMaxAttemptsExceededError(
                    oid.hex(), "the creating task's max_retries is exhausted")
            if spec["retries"] > 0:
                spec["retries"] -= 1
            spec["attempt"] += 1
            if revived:
                del self.lineage_objs[oid]
                self.owned[oid] = o
            # the spec leaves the lineage table while it re-runs but keeps its argument
            # lineage refs (_largs); _complete puts it back
            del self.lineage[tid]
            self.task_specs[tid] = spec
            for i in range(spec["nret"]):
                r = self.owned.get(object_id_for_return(tid, i + 1))
                if r is not None:
                    r.ready = False
                    self._ready_owned.discard(object_id_for_return(tid, i + 1))
                    r.inline = None
                    r.in_store = False
                    r.node = None
                    r.recon += 1
            args = [a for a, owner, inline in spec["args"][1]
                    if owner == self.addr and inline is None]
        # lost or freed arguments are re-created first (recursively through their own
        # lineage); dependency resolution waits for them
        from ray_amd.object_ref import ObjectRef

        holders = []
        for a in args:
            with self.lock:
                ao = self.owned.get(a)
                freed = ao is None and a in self.lineage_objs
                check = ao is not None and ao.ready and ao.in_store
                anode = ao.node if ao is not None else None
            if freed or (check and not self._copy_available(a, anode)):
                err = self._reconstruct(a, anode)
                if err is not None:
                    self._fail_task(spec, err)
                    return None
            if a in self.owned:  # pinned until the re-run completes
                holders.append(ObjectRef(a, self.addr, _cw_obj=self))
        spec["_holders"] = holders
        self.task_events.append((tid, spec.get("name"), time.time(), None, None, None,
                                 "PENDING_ARGS_AVAIL", P.NORMAL_TASK, self.job_id,
                                 spec["attempt"], None))
        self._resolve_and_schedule(spec)
        return None

    def _copy_available(self, oid, node) -> bool:
        """Non-blocking check (runs on the dispatcher too): only a local copy can be
        verified; an argument on another node is assumed present — if it is not, the
        re-executed task's worker reports it through recover_object, recursively."""
        if node is None or node == self.node_hex:
            return self.store is not None and self.store.contains(oid)
        return True

    # ------------------------------------------------------------------ manual free
    def free_objects(self, oids, local_only=False):
        """ray.internal.free: drop the stored value of each object now, whatever its
        reference count. Later gets raise ObjectFreedError; freed objects are never
        reconstructed. Objects owned elsewhere are freed by their owner (unless
        local_only: then only this node's store copy goes)."""
        by_owner: dict = {}
        for oid in oids:
            with self.lock:
                owned = oid in self.owned
                e = self.refs.get(oid)
                owner = e[1] if e else None
            if owned:
                self._free_owned(oid)
            elif local_only or owner is None:
                if self.store is not None:
                    try:
                        self.store.delete(oid)
                    except Exception:
                        pass
            else:
                by_owner.setdefault(owner, []).append(oid)
        for owner, lst in by_owner.items():
            self.send(owner, (P.REQ, 0, "free_objects_owned", (lst,)))

    def _free_owned(self, oid):
        from ray_amd.exceptions import ObjectFreedError

        data = ser.serialize_error(ObjectFreedError(oid.hex())).to_bytes()
        with self.lock:
            o = self.owned.get(oid)
            if o is None:
                return
            tid = o.task_id
            was_ready = o.ready
            in_store, node = o.in_store, o.node
            o.task_id = None  # freed values are not reconstructed
            if was_ready:
                o.inline, o.in_store, o.node = data, False, None
        if not was_ready:
            self._mark_ready(oid, inline=data)
        elif in_store:
            self._delete_stored(oid, node)
        with self.lock:
            self._drop_lineage_if_unused(tid)

    def _rpc_free_objects_owned(self, conn, rid, oids):
        for oid in oids:
            self._free_owned(oid)
        self._reply(conn, rid, True, None)

    def _rpc_recover_object(self, conn, rid, oid, failed_node):
        """A borrower could not fetch `oid`: reconstruct it, reply once it is ready."""
        err = self._reconstruct(oid, failed_node)
        if err is not None:
            self._reply(conn, rid, True, (False, err))
            return

        def done(_oid):
            self._reply(conn, rid, True, (True, None))

        if self._on_ready(oid, done):
            done(oid)

    def _value_of_once(self, oid: bytes, anchor: str | None):
        with self.lock:
            o = self.owned.get(oid)
            if o is not None:
                inline, in_store = o.inline, o.in_store
                owner = self.addr
                node = o.node
                o.accessed = True
            else:
                r = self.remote.get(oid)
                inline = r.inline if r else None
                in_store = inline is None
                node = r.node if r else None
                e = self.refs.get(oid)
                owner = e[1] if e else None
                if r is not None and r.state == 3:
                    raise r.error
        if inline is not None:
            buf = inline
        else:
            buf = self.store.get_buffer(oid)
            if buf is None and node is not None and node != self.node_hex:
                buf = self._fetch_remote(oid, node)
            if buf is None:
                raise _CopyLost(node)
        kind, value = ser.deserialize(buf, ser.DeserializeContext(anchor=owner))
        if kind == ser.KIND_ERROR:
            if isinstance(value, RayTaskError):
                raise value.as_instanceof_cause()
            raise value
        return value

    def wait_refs(self, oids, num_returns, timeout):
        """Returns the list of ready oids (at least num_returns unless timeout)."""
        # Owned objects are polled under the readiness condition variable (notified by
        # _mark_ready); only borrowed objects need per-object owner callbacks.
        owned = self.owned
        ids = oids if isinstance(oids, (set, frozenset)) else set(oids)
        with self.lock:
            done = ids & self._ready_owned  # set algebra: C speed per ref
            if len(done) >= num_returns:
                return done
            rest = ids - done
            owned_pending = rest & owned.keys()
            remote_pending = rest - owned_pending if len(owned_pending) != len(rest) else ()
        cv = self._ready_cv

        def remote_hit(oid):
            with self.lock:
                done.add(oid)
                cv.notify_all()

        registered = []
        for oid in remote_pending:
            if self._on_ready(oid, remote_hit):
                done.add(oid)
            else:
                registered.append(oid)
        if len(done) >= num_returns or (timeout is not None and timeout <= 0):
            self._drop_waiter(registered, remote_hit)
            return self._collect_ready(done, owned_pending, num_returns)
        deadline = None if timeout is None else time.monotonic() + timeout
        blocked = self._maybe_notify_blocked()
        # A wake-up looks only at the objects that became ready since the previous one (the
        # ready log), not at every pending ref: wait() on 1k refs was quadratic.
        try:
            with self.lock:
                # re-check what became ready (or was freed: counts as ready) since the
                # first look, with set algebra instead of a per-ref loop
                done |= owned_pending & self._ready_owned
                pend = owned_pending - done
                gone = pend - self.owned.keys()
                if gone:
                    done |= gone
                    pend -= gone
                seen = self._ready_seq
                log = self._ready_log
                while len(done) < num_returns and not self.exiting:
                    rem = None if deadline is None else deadline - time.monotonic()
                    if rem is not None and rem <= 0:
                        break
                    # every ready object bumps _ready_seq, so num_returns - len(done) more
                    # is the earliest point at which this wait can be satisfied (borrowed
                    # refs notify directly through remote_hit)
                    target = self._ready_seq + (num_returns - len(done))
                    self._wake_targets.append(target)
                    try:
                        cv.wait(rem if rem is not None else 1.0)
                    finally:
                        self._wake_targets.remove(target)
                    new = self._ready_seq - seen
                    seen = self._ready_seq
                    if new > len(log):  # log wrapped: rescan what is left
                        hit = {oid for oid in pend if (self.owned.get(oid) is None or
                                                       self.owned[oid].ready)}
                    else:  # only the objects that became ready since the last look
                        hit = {log[-1 - i] for i in range(new)} & pend
                    if hit:
                        done |= hit
                        pend -= hit
        finally:
            if blocked:
                self._notify_unblocked()
            self._drop_waiter(registered, remote_hit)
        return set(done)

    def _collect_ready(self, done, owned_pending, num_returns):
        with self.lock:
            done = set(done) | (owned_pending & self._ready_owned)
            done |= owned_pending - self.owned.keys()  # freed meanwhile: ready
        return done

    def _drop_waiter(self, oids, cb):
        """Unregister a finished waiter so callbacks do not pile up on pending objects."""
        with self.lock:
            for oid in oids:
                o = self.owned.get(oid)
                lst = o.callbacks if o is not None else None
                if lst is None:
                    r = self.remote.get(oid)
                    lst = r.callbacks if r is not None else None
                if lst:
                    try:
                        lst.remove(cb)
                    except ValueError:
                        pass

    def get_objects(self, refs, timeout=None):
        oids = [r._id for r in refs]
        uniq = list(dict.fromkeys(oids))
        ready = self.wait_refs(uniq, len(uniq), timeout)
        if len(ready) < len(uniq):
            raise GetTimeoutError(f"Get timed out: {len(uniq) - len(ready)} objects not ready "
                                  f"after {timeout}s")
        out = []
        for r in refs:
            out.append(self._value_of(r._id, None))
        return out

    def as_concurrent_future(self, ref):
        import concurrent.futures

        fut = concurrent.futures.Future()

        def done(oid, ref=ref):
            try:
                v = self._value_of(oid, None)
            except BaseException as e:  # noqa: BLE001
                if not fut.done():
                    fut.set_exception(e)
                return
            if not fut.done():
                fut.set_result(v)

        def cb(oid):
            threading.Thread(target=done, args=(oid,), daemon=True).start()

        if self._on_ready(ref._id, cb):
            done(ref._id)
        return fut

    def _maybe_notify_blocked(self) -> bool:
        if self.mode != "worker" or getattr(self.current_task, "tid", None) is None:
            return False
        lid = getattr(self.current_task, "lease_id", None)
        if lid is None:
            return False
        with self.lock:
            self.blocked_depth += 1
            first = self.blocked_depth == 1
        if first:
            self.notify_raylet("notify_blocked", self.worker_id)
            if PIPELINE_DEPTH > 1:
                # tasks pipelined behind this one go back to their owners: the blocked task
                # may be waiting for one of them
                self._requeue_to_owner(self._take_queued())
        return True

    def _notify_unblocked(self):
        with self.lock:
            self.blocked_depth -= 1
            last = self.blocked_depth == 0
        if last:
            self.notify_raylet("notify_unblocked", self.worker_id)

    # ------------------------------------------------------------------ functions
    def export(self, obj) -> bytes:
        """Export a function/class to the cluster KV; returns its key."""
        key = getattr(obj, "__ray_amd_key__", None)
        if key is not None and key in self.exported:
            return key
        data = cloudpickle.dumps(obj)
        key = hashlib.blake2b(data, digest_size=16).digest()
        if key not in self.exported:
            # Synchronous: a cached lease pushes the task straight to a worker, whose
            # kv_get must not overtake this put on the raylet.
            self.call_raylet("kv_put", "fn", key, data, True)
            self.exported.add(key)
            self.fn_cache[key] = obj
        return key

    def _load_function(self, key):
        fn = self.fn_cache.get(key)
        if fn is None:
            data = self.call_raylet("kv_get", "fn", key)
            if data is None:
                raise RuntimeError(f"function {key.hex()} not found in cluster KV")
            fn = cloudpickle.loads(data)
            self.fn_cache[key] = fn
        return fn

    # ------------------------------------------------------------------ args
    def _encode_args(self, args, kwargs):
        """Top-level ObjectRef args are resolved by the executor; everything else is
        serialized in one blob (large blobs go to the store)."""
        from ray_amd.object_ref import ObjectRef

        ref_args = []
        holders = []
        if any(isinstance(a, ObjectRef) for a in args) or \
                any(isinstance(v, ObjectRef) for v in kwargs.values()):
            a2 = []
            for a in args:
                if isinstance(a, ObjectRef):
                    a2.append(_ArgRef(len(ref_args)))
                    ref_args.append(self._ref_desc(a))
                    holders.append(a)
                else:
                    a2.append(a)
            k2 = {}
            for k, v in kwargs.items():
                if isinstance(v, ObjectRef):
                    k2[k] = _ArgRef(len(ref_args))
                    ref_args.append(self._ref_desc(v))
                    holders.append(v)
                else:
                    k2[k] = v
            args, kwargs = a2, k2
        if not args and not kwargs:
            return (None, ref_args), holders
        put_oid = object_id_for_put(self._current_task_id(), self._bump_put())
        sobj = ser.serialize((args, kwargs), put_oid)
        holders.extend(sobj.refs)
        if sobj.total > ARGS_INLINE_MAX or sobj.gpu:
            ref = self.put_serialized_object(put_oid, sobj)
            holders.append(ref)
            return (("s", ref._id, self.addr), ref_args), holders
        return (sobj.to_bytes(), ref_args), holders

    def _bump_put(self):
        with self.lock:
            self.put_index += 1
            return self.put_index

    def _ref_desc(self, ref):
        oid = ref._id
        with self.lock:
            o = self.owned.get(oid)
            if o is not None and o.ready and o.inline is not None:
                o.accessed = True  # inlined into a task: the receiver reads it
                return (oid, ref._owner, o.inline)
        return (oid, ref._owner, None)

    def _decode_args(self, encoded, owner_addr):
        blob, ref_args = encoded
        vals = []
        if ref_args:
            from ray_amd.object_ref import ObjectRef

            need = []
            for oid, owner, inline in ref_args:
                if inline is not None:
                    vals.append(("v", inline, owner))
                else:
                    ref = ObjectRef(oid, owner, _cw_obj=self)
                    need.append(ref)
                    vals.append(("r", ref, owner))
            if need:
                self.wait_refs([r._id for r in need], len(need), None)
            res = []
            for kind, x, owner in vals:
                if kind == "v":
                    k, v = ser.deserialize(x, ser.DeserializeContext(anchor=owner_addr))
                    if k == ser.KIND_ERROR:
                        raise v.as_instanceof_cause() if isinstance(v, RayTaskError) else v
                    res.append(v)
                else:
                    res.append(self._value_of(x._id, owner_addr))
            vals = res
        if blob is None:
            args, kwargs = [], {}
        else:
            if isinstance(blob, tuple):
                _, oid, owner = blob
                buf = self.store.get_buffer(oid)
                if buf is None:
                    raise ObjectLostError(oid.hex())
            else:
                buf = blob
            _, (args, kwargs) = ser.deserialize(buf, ser.DeserializeContext(anchor=owner_addr))
        if ref_args:
            args = [vals[a.i] if isinstance(a, _ArgRef) else a for a in args]
            kwargs = {k: (vals[v.i] if isinstance(v, _ArgRef) else v) for k, v in kwargs.items()}
        return args, kwargs

    # ------------------------------------------------------------------ normal tasks
    def new_task_id(self) -> bytes:
        with self.lock:
            self.task_counter += 1
            c = self.task_counter
        return self.task_id_base + c.to_bytes(4, "little")

    def submit_task(self, fn_key, args, kwargs, opts: dict, name: str):
        """Submit a normal task; returns list of ObjectRefs (or a generator)."""
        from ray_amd.object_ref import ObjectRef, ObjectRefGenerator

        tid = self.new_task_id()
        nret = opts.get("num_returns", 1)
        dynamic = nret == "dynamic"
        if dynamic:
            nret = 1
        streaming = nret == "streaming"
        encoded, holders = self._encode_args(args, kwargs)
        spec = {
            "tid": tid, "type": P.NORMAL_TASK, "fn": fn_key, "args": encoded,
            "nret": -1 if streaming else nret, "owner": self.addr, "name": name,
            "resources": opts["resources"], "strategy": opts.get("strategy"),
            "retries": opts.get("max_retries", 3), "retry_exc": opts.get("retry_exceptions", False),
            "runtime_env": self._export_renv(opts.get("runtime_env")), "attempt": 0,
            "job": self.job_id, "dynamic": dynamic, "ns": self.namespace,
        }
        if opts.get("max_calls"):
            spec["max_calls"] = int(opts["max_calls"])
        if opts.get("enable_task_events", True) is False:
            spec["no_events"] = True  # kept out of the task-event stream / timeline
        bp = int(opts.get("_generator_backpressure_num_objects") or 0)
        if streaming and bp > 0:
            spec["gen_bp"] = bp
        refs = []
        with self.lock:
            if streaming:
                self.streams[tid] = _Stream(spec.get("gen_bp", 0))
            else:
                for i in range(nret):
                    oid = object_id_for_return(tid, i + 1)
                    self.owned[oid] = _Owned(tid)
            self.task_specs[tid] = spec
        self._note_child(tid)
        if not streaming:
            refs = [ObjectRef(object_id_for_return(tid, i + 1), self.addr, _cw_obj=self)
                    for i in range(nret)]
        spec["_holders"] = holders
        if _tracing.ENABLED:
            _tracing.inject(spec, "function")
        if not spec.get("no_events"):
            self.task_events.append((tid, name, time.time(), None, None, None,
                                     "PENDING_NODE_ASSIGNMENT", P.NORMAL_TASK, self.job_id, 0,
                                     None))
        if self.local_mode:
            self._run_local(spec)
        else:
            self._resolve_and_schedule(spec)
        if streaming:
            return ObjectRefGenerator(tid, self, self.addr)
        return refs

    def _resolve_and_schedule(self, spec):
        """Owner-side dependency resolution: wait for owned pending args."""
        pending = []
        for oid, owner, inline in spec["args"][1]:
            if owner == self.addr and inline is None:
                with self.lock:
                    o = self.owned.get(oid)
                    if o is not None and not o.ready:
                        pending.append(oid)
        if not pending:
            self._inline_ready_args(spec)
            self._schedule(spec)
            return
        remaining = [len(pending)]
        lock = threading.Lock()

        def dep_ready(_oid):
            with lock:
                remaining[0] -= 1
                done = remaining[0] == 0
            if done:
                self._inline_ready_args(spec)
                self._schedule(spec)

        for oid in pending:
            if self._on_ready(oid, dep_ready):
                dep_ready(oid)

    def _inline_ready_args(self, spec):
        blob, ref_args = spec["args"]
        if not ref_args:
            return
        new = []
        for oid, owner, inline in ref_args:
            if inline is None and owner == self.addr:
                with self.lock:
                    o = self.owned.get(oid)
                    if o is not None and o.ready and o.inline is not None:
                        inline = o.inline
                        o.accessed = True
            new.append((oid, owner, inline))
        spec["args"] = (blob, new)

    @staticmethod
    def _sched_key(spec):
        res = spec["resources"]
        st = spec.get("strategy")
        renv = spec.get("runtime_env")
        return (tuple(sorted(res.items())), repr(st), repr(renv) if renv else None)

    def _schedule(self, spec):
        key = self._sched_key(spec)
        with self.lock:
            if spec["tid"] in self.cancelled:
                cancelled = True
            else:
                cancelled = False
                self.sched_queues[key].append(spec)
        if cancelled:
            self._fail_task(spec, TaskCancelledError(spec["tid"].hex()))
            return
        self._pump(key)

    @staticmethod
    def _pipelinable(spec) -> bool:
        # never queued behind another task: tasks that retire their worker (max_calls),
        # streaming generators and tasks without retries (a worker death would fail a task
        # that never ran)
        return not spec.get("max_calls") and spec["nret"] != -1 and spec["retries"] != 0

    def _saturated(self, key, now) -> bool:
        t = self._lease_wait_t.get(key)
        return t is not None and self.pending_leases[key] > 0 and now - t > PIPELINE_AFTER_S

    def _pump(self, key):
        to_send = []
        request = 0
        with self.lock:
            q = self.sched_queues.get(key)
            if not q:
                return
            leases = self.leases.get(key, ())
            for lease in leases:
                while q and not lease.inflight:
                    spec = q.popleft()
                    lease.inflight[spec["tid"]] = spec
                    self.task_lease[spec["tid"]] = lease
                    to_send.append((lease, spec))
            if q and PIPELINE_DEPTH > 1 and leases and \
                    self._saturated(key, time.monotonic()):
                for lease in leases:
                    while q and len(lease.inflight) < PIPELINE_DEPTH and \
                            self._pipelinable(q[0]) and \
                            all(self._pipelinable(sp) for sp in lease.inflight.values()):
                        spec = q.popleft()
                        lease.inflight[spec["tid"]] = spec
                        self.task_lease[spec["tid"]] = lease
                        to_send.append((lease, spec))
                        self.pipeline_stats["pipelined"] += 1
            if q:
                want = min(len(q), MAX_PENDING_LEASES_PER_KEY) - self.pending_leases[key]
                if want > 0:
                    request = want
                    if self.pending_leases[key] == 0:
                        self._lease_wait_t[key] = time.monotonic()
                    self.pending_leases[key] += want
        for lease, spec in to_send:
            self._push_task(lease.addr, spec, lease.lease_id)
        for _ in range(request):
            self._request_lease(key)

    def _steal_for(self, key):
        """A lease of ``key`` went idle with nothing queued: take back one pipelined task
        that is still waiting in a busy worker's queue (the worker answers with a requeue
        reply if it has not started it)."""
        with self.lock:
            if self.sched_queues.get(key):
                return
            for lease in self.leases.get(key, ()):
                if len(lease.inflight) > 1:
                    tid = next(reversed(lease.inflight))
                    if tid in self._stealing:
                        continue
                    self._stealing.add(tid)
                    self.pipeline_stats["steals"] += 1
                    addr = lease.addr
                    break
            else:
                return
        self.send(addr, (P.STEAL, tid))

    def _push_task(self, addr, spec, lease_id):
        wire = {k: v for k, v in spec.items() if not k.startswith("_")}
        wire["lease_id"] = lease_id
        if not self.send(addr, (P.TASK, wire)):
            self._on_worker_lost(addr)

    def _request_lease(self, key):
        res, strat_repr, _ = key
        with self.lock:
            q = self.sched_queues.get(key)
            sample = q[0] if q else None
        if sample is None:
            with self.lock:
                self.pending_leases[key] -= 1
            return
        req = {
            "resources": sample["resources"], "strategy": sample.get("strategy"),
            "runtime_env": sample.get("runtime_env"), "owner": self.addr, "job": self.job_id,
            "name": sample.get("name"), "retriable": sample.get("retries", 0) != 0,
        }

        def on_lease(ok, value, key=key):
            with self.lock:
                self.pending_leases[key] -= 1
                # a grant: the node had room; the wait clock restarts for what is still out
                self._lease_wait_t[key] = time.monotonic()
            if not ok:
                err = value if isinstance(value, BaseException) else RuntimeError(str(value))
                with self.lock:
                    q = self.sched_queues.pop(key, collections.deque())
                for spec in q:
                    self._fail_task(spec, err)
                return
            lease = _Lease(value["addr"], value["lease_id"], key, value.get("gpu_ids"),
                           value.get("worker_id"))
            with self.lock:
                self.leases[key].append(lease)
            self._pump(key)
            if not lease.inflight and PIPELINE_DEPTH > 1:
                # a fresh worker with nothing queued: take back a task pipelined behind a
                # running one elsewhere (it would otherwise wait for that task to finish)
                self._steal_for(key)
            # nothing left to run on it: give it back
            self._maybe_return_lease(lease, force=False)

        self.call_async(self.raylet_addr, "request_lease", (req,), on_lease)

    def _maybe_return_lease(self, lease, force):
        with self.lock:
            if lease.inflight:
                return
            q = self.sched_queues.get(lease.key)
            if q and not force:
                return
            if not force and time.monotonic() - lease.idle_since < LEASE_IDLE_S:
                return
            try:
                self.leases[lease.key].remove(lease)
            except ValueError:
                return
        self.notify_raylet("return_lease", lease.lease_id, False)

    def _reap_idle_leases(self):
        now = time.monotonic()
        for key, ls in list(self.leases.items()):
            for lease in list(ls):
                if not lease.inflight and now - lease.idle_since >= LEASE_IDLE_S:
                    self._maybe_return_lease(lease, force=False)

    def _on_task_reply(self, conn, msg):
        _, tid, returns, extra = msg
        evs = extra.get("events")
        if evs:
            self.task_events.extend(evs)
        if extra.get("requeue"):  # a pipelined task handed back unstarted
            self._on_requeue(tid)
            return
        if self._stealing:
            self._stealing.discard(tid)  # finished before the steal reached it
        with self.lock:
            spec = self.task_specs.get(tid)
        if spec is None:
            # unknown (cancelled / duplicate): drop store results
            for oid, kind, payload, contained in returns:
                if kind == P.RET_STORE:
                    self._delete_stored(oid, extra.get("node"))
            return
        if spec["type"] == P.ACTOR_TASK:
            self._on_actor_task_reply(spec, returns, extra)
            return
        lease = None
        retire = False
        with self.lock:
            lease = self.task_lease.pop(tid, None)
            if lease is not None:
                lease.inflight.pop(tid, None)
                lease.idle_since = time.monotonic()
                if extra.get("worker_exit"):  # max_calls reached: retire that worker
                    try:
                        self.leases[lease.key].remove(lease)
                        retire = True
                    except ValueError:
                        pass
        if retire:
            self.notify_raylet("return_lease", lease.lease_id, True)
        # application-level retry
        if extra.get("app_error") and self._should_retry_exc(spec, extra.get("exc_type")):
            for oid, kind, payload, contained in returns:
                if kind == P.RET_STORE:
                    self._delete_stored(oid, extra.get("node"))
            spec["retries"] -= 1 if spec["retries"] > 0 else 0
            spec["attempt"] += 1
            self._schedule(spec)
        else:
            self._complete(spec, returns, extra)
        if lease is not None:
            self._pump(lease.key)
            if not lease.inflight and PIPELINE_DEPTH > 1:
                self._steal_for(lease.key)

    def _on_requeue(self, tid):
        with self.lock:
            self.pipeline_stats["requeued"] += 1
            self._stealing.discard(tid)
            lease = self.task_lease.pop(tid, None)
            spec = self.task_specs.get(tid)
            if lease is not None:
                lease.inflight.pop(tid, None)
                if not lease.inflight:
                    lease.idle_since = time.monotonic()
            if spec is None:
                return
            key = self._sched_key(spec)
            self.sched_queues[key].appendleft(spec)
        self._pump(key)
        if lease is not None:
            self._pump(lease.key)

    def _should_retry_exc(self, spec, exc_type_name):
        re = spec.get("retry_exc")
        if not re or spec["retries"] == 0:
            return False
        if re is True:
            return True
        names = {getattr(c, "__name__", str(c)) for c in re}
        return exc_type_name in names

    def _complete(self, spec, returns, extra, call_finished=False):
        from ray_amd.object_ref import ObjectRef

        tid = spec["tid"]
        with self.lock:
            self.task_specs.pop(tid, None)
        # a failed call of a handle-less actor may be the one it was waiting for
        # (connection loss, the lost-task fallback timer, a dead actor); a reply already
        # went through _actor_call_finished (call_finished)
        if spec["type"] == P.ACTOR_TASK and not call_finished and \
                self._actor_call_finished(spec) and not self._stopped:
            self.notify_raylet("actor_out_of_scope", spec["actor_id"])
        if spec["nret"] == -1:
            st = self.streams.get(tid)
            if st is not None:
                with self.lock:
                    st.done = True
                    st.total = extra.get("num_items")
                    if returns:
                        oid, kind, payload, contained = returns[0]
                        self.owned[oid] = _Owned(tid)
                        st.error_ref = ObjectRef(oid, self.addr, _cw_obj=self)
                    else:
                        st.error_ref = None
                if returns:
                    self._mark_ready(returns[0][0], inline=returns[0][2])
                self._wake_stream(tid)
            return
        node = extra.get("node")
        stored = False
        for oid, kind, payload, contained in returns:
            pins = None
            if contained:
                for c_oid, c_owner in contained:
                    self._add_borrow_credit(c_oid, c_owner)
                pins = [ObjectRef(c_oid, c_owner, _cw_obj=self) for c_oid, c_owner in contained]
            if kind == P.RET_INLINE:
                self._mark_ready(oid, inline=payload, contained=pins, size=len(payload))
            else:
                stored = True
                self._mark_ready(oid, in_store=True, contained=pins, size=payload, node=node)
        with self.lock:
            if (stored and spec["type"] == P.NORMAL_TASK and not spec.get("dynamic")
                    and any(object_id_for_return(tid, i + 1) in self.owned
                            for i in range(spec["nret"]))):
                # keep the spec as lineage while its stored returns are referenced
                # (inline returns can never be lost). It names its stored arguments by
                # id only: their values are freed with their last in-scope ref.
                self._add_lineage(tid, spec)
            elif "_largs" in spec:  # a re-run whose lineage is no longer needed
                for t in self._release_lineage_args(spec):
                    self._drop_lineage_if_unused(t)
        holders = spec.pop("_holders", None)
        del holders  # may free argument values (outside the lock's critical section)

    def _add_lineage(self, tid, spec):
        """(lock held) Record a finished task's spec as lineage; bounded by count and bytes."""
        if "_largs" not in spec:  # first completion (a re-run keeps its refs)
            largs = []
            nbytes = 256
            blob = spec["args"][0]
            if isinstance(blob, (bytes, bytearray, memoryview)):
                nbytes += len(blob)
            for a, owner, inline in spec["args"][1]:
                if inline is not None:
                    nbytes += len(inline)
                elif owner == self.addr:
                    o = self.owned.get(a) or self.lineage_objs.get(a)
                    if o is not None:
                        o.lineage_refs += 1
                        largs.append(a)
            spec["_largs"] = largs
            spec["_lbytes"] = nbytes
            self.lineage_bytes += nbytes
        self.lineage[tid] = spec
        self.lineage.move_to_end(tid)
        while len(self.lineage) > 1 and (len(self.lineage) > LINEAGE_MAX
                                         or self.lineage_bytes > LINEAGE_MAX_BYTES):
            old_tid, old = self.lineage.popitem(last=False)
            self.lineage_evicted.add(old_tid)
            for t in self._release_lineage_args(old):
                self._drop_lineage_if_unused(t)
            # freed returns of the evicted task can no longer be re-created
            for i in range(max(old["nret"], 0)):
                self.lineage_objs.pop(object_id_for_return(old_tid, i + 1), None)

    def _fail_task(self, spec, exc):
        sobj = ser.serialize_error(exc)
        data = sobj.to_bytes()
        tid = spec["tid"]
        with self.lock:
            self.task_specs.pop(tid, None)
        # a failed call of a handle-less actor may be the one it was waiting for
        # (connection loss, the lost-task fallback timer, a dead actor)
        if spec["type"] == P.ACTOR_TASK and self._actor_call_finished(spec) and \
                not self._stopped:
            self.notify_raylet("actor_out_of_scope", spec["actor_id"])
        if spec["nret"] == -1:
            st = self.streams.get(tid)
            if st is not None:
                from ray_amd.object_ref import ObjectRef

                oid = object_id_for_return(tid, 0x7FFFFFFF)
                with self.lock:
                    self.owned[oid] = _Owned(tid)
                    st.error_ref = ObjectRef(oid, self.addr, _cw_obj=self)
                    st.done = True
                self._mark_ready(oid, inline=data)
                self._wake_stream(tid)
            return
        n = spec["nret"] if spec["type"] != P.ACTOR_CREATION_TASK else 0
        for i in range(n):
            self._mark_ready(object_id_for_return(tid, i + 1), inline=data)
        if "_largs" in spec:  # a failed re-run: its lineage is gone
            with self.lock:
                for t in self._release_lineage_args(spec):
                    self._drop_lineage_if_unused(t)
        spec.pop("_holders", None)

    def _on_worker_lost(self, addr):
        lost = []
        queued = []  # pipelined behind the running task: never started on that worker
        with self.lock:
            for key, ls in list(self.leases.items()):
                for lease in list(ls):
                    if lease.addr == addr:
                        ls.remove(lease)
                        specs = list(lease.inflight.values())
                        lost.extend(specs[:1])
                        queued.extend(specs[1:])
                        for t in lease.inflight:
                            self.task_lease.pop(t, None)
                            self._stealing.discard(t)
                        lease.inflight.clear()
        for spec in queued:  # rescheduled as they are: no retry consumed
            self._schedule(spec)
        if not lost:
            return

        def with_cause(ok, cause, lost=lost):
            # the raylet tells us whether IT killed the worker (memory monitor)
            oom = ok and isinstance(cause, str) and cause.startswith("oom:")
            retry_ok = True
            msg = ""
            if oom:
                _, flag, msg = cause.split(":", 2)
                retry_ok = flag == "retry"  # the kill policy's verdict
            for spec in lost:
                if spec["retries"] != 0 and retry_ok:
                    if spec["retries"] > 0:
                        spec["retries"] -= 1
                    spec["attempt"] += 1
                    self._schedule(spec)
                elif oom:
                    self._fail_task(spec, OutOfMemoryError(msg))
                else:
                    self._fail_task(spec, WorkerCrashedError())

        self.call_async(self.raylet_addr, "death_cause", (addr,), with_cause)

    # ------------------------------------------------------------------ streaming
    def _on_stream_item(self, conn, msg):
        tid, index, ret = msg[1], msg[2], msg[3]
        node = msg[4] if len(msg) > 4 else None
        from ray_amd.object_ref import ObjectRef

        oid, kind, payload, contained = ret
        st = self.streams.get(tid)
        if st is None:
            if kind == P.RET_STORE:
                self._delete_stored(oid, node)
            return
        with self.lock:
            self.owned[oid] = _Owned(tid)
        ref = ObjectRef(oid, self.addr, _cw_obj=self)
        for a, b in contained or ():
            self._add_borrow_credit(a, b)
        pins = [ObjectRef(a, b, _cw_obj=self) for a, b in contained] if contained else None
        if kind == P.RET_INLINE:
            self._mark_ready(oid, inline=payload, contained=pins)
        else:
            self._mark_ready(oid, in_store=True, contained=pins, size=payload, node=node)
        with self.lock:
            st.items[index] = ref
            st.conn = conn
        self._wake_stream(tid)

    def _wake_stream(self, tid):
        with self.lock:
            self._stream_cv().notify_all()

    def _stream_cv(self):
        cv = getattr(self, "_scv", None)
        if cv is None:
            self._scv = cv = threading.Condition(self.lock)
        return cv

    def next_stream_item(self, tid, index, timeout):
        cv = self._stream_cv()
        with self.lock:
            st = self.streams.get(tid)
            if st is None:
                return None
            while True:
                if index in st.items:
                    st.consumed = max(st.consumed, index + 1)
                    if st.bp and st.conn is not None:  # let a throttled generator go on
                        self.io.send(st.conn, _dumps((P.STREAM_ACK, tid, st.consumed)))
                    return st.items.pop(index)
                if st.done:
                    if st.total is not None and index < st.total:
                        pass  # item message still in flight
                    else:
                        if st.error_ref is not None:
                            r, st.error_ref = st.error_ref, None
                            return r
                        return None
                cv.wait(0.5)

    def stream_completed_ref(self, tid):
        with self.lock:
            st = self.streams.get(tid)
            return st is not None and st.done

    def drop_stream(self, tid):
        with self.lock:
            self.streams.pop(tid, None)

    # ------------------------------------------------------------------ cancellation
    def cancel(self, ref, force=False, recursive=True):
        """ray.cancel (reference: python/ray/_raylet.pyx:2357 kill_main_task,
        src/ray/core_worker/core_worker.cc:3821 HandleCancelTask). A queued task fails
        with TaskCancelledError at once; a running one is interrupted where it runs: the
        worker's main thread gets a real SIGINT (time.sleep, socket reads, ray.get and
        other blocking calls return at once with KeyboardInterrupt -> TaskCancelledError),
        an async actor's coroutine is cancelled on its loop, and force=True kills the
        worker process. recursive=True also cancels the tasks the cancelled task submitted.
        A non-owner forwards the request to the owner."""
        tid = ref._id[:16]
        with self.lock:
            spec = self.task_specs.get(tid)
            known = spec is not None
        if known and force and spec["type"] == P.ACTOR_TASK:
            # reference: core_worker.cc HandleCancelTask / CancelTask rejects it — killing
            # the actor process would take its state and every other in-flight call along
            raise ValueError("force=True is not supported for actor tasks.")
        if not known:
            owner = getattr(ref, "_owner", None)
            if owner and owner != self.addr:
                self.send(owner, (P.REQ, 0, "cancel_request", (tid, force, recursive)))
            return
        self._cancel_tid(tid, force, recursive)

    def _rpc_cancel_request(self, conn, rid, tid, force, recursive=True):
        """A borrower asked the owner to cancel one of its tasks."""
        self._cancel_tid(tid, force, recursive)
        if rid:
            self._reply(conn, rid, True, None)

    def _cancel_tid(self, tid, force=False, recursive=True):
        with self.lock:
            spec = self.task_specs.get(tid)
            if spec is None:
                return
            self.cancelled.add(tid)
            # still queued locally?
            for key, q in self.sched_queues.items():
                if spec in q:
                    q.remove(spec)
                    queued = True
                    break
            else:
                queued = False
            lease = self.task_lease.get(tid)
        if queued:
            self._fail_task(spec, TaskCancelledError(tid.hex()))
            return
        if spec["type"] == P.ACTOR_TASK:
            force = False  # a forwarded force=True never kills an actor process
        msg = (P.REQ, 0, "cancel_task", (tid, force, recursive))
        if spec["type"] == P.ACTOR_TASK:
            ac = self.actors.get(spec["actor_id"])
            if ac is not None and ac.addr:
                self.send(ac.addr, msg)
            return
        if lease is not None:
            self.send(lease.addr, msg)

    def _rpc_cancel_task(self, conn, rid, tid, force, recursive=True):
        with self.lock:
            self.cancelled.add(tid)
            th = self.running.get(tid)
            kids = list(self._children.get(tid, ())) if recursive else []
            atask = self._async_tasks.get(tid)
        for k in kids:  # tasks this task submitted (this worker owns them)
            try:
                self._cancel_tid(k, force, recursive)
            except Exception:
                pass
        if atask is not None:  # async actor method: never force-killed (see cancel)
            loop, task = atask
            loop.call_soon_threadsafe(task.cancel)
        elif th is not None:
            if force:
                os._exit(1)
            self._interrupt_thread(th)
        if rid:
            self._reply(conn, rid, True, None)

    def _interrupt_thread(self, th: int):
        """Deliver the cancellation to the thread running the task: a real SIGINT for the
        main thread (interrupts blocking C calls), an asynchronous exception otherwise
        (threaded actors: raised at the thread's next bytecode)."""
        import signal

        if self._sigint_installed and th == threading.main_thread().ident:
            signal.pthread_kill(th, signal.SIGINT)
        else:
            _raise_in_thread(th, KeyboardInterrupt)

    def install_cancel_handler(self):
        """Worker processes: SIGINT raises KeyboardInterrupt in the main thread only while
        a cancelled task's user code runs there; stray or early signals (argument
        deserialisation, between tasks) are ignored — the pre-call check catches those."""
        import signal

        def _on_sigint(signum, frame):
            tid = getattr(self.current_task, "tid", None)
            if self._main_interruptible and tid is not None and tid in self.cancelled:
                raise KeyboardInterrupt

        try:
            signal.signal(signal.SIGINT, _on_sigint)
            self._sigint_installed = True
        except ValueError:  # not the main thread
            self._sigint_installed = False

    def _note_child(self, tid):
        parent = getattr(self.current_task, "tid", None)
        if parent is not None:
            with self.lock:
                self._children.setdefault(parent, []).append(tid)

    # ------------------------------------------------------------------ actors (caller)
    def create_actor(self, actor_id: bytes, cls_key, args, kwargs, opts: dict, cls_name: str,
                     method_meta: dict):
        encoded, holders = self._encode_args(args, kwargs)
        spec = {
            "tid": self.new_task_id(), "type": P.ACTOR_CREATION_TASK, "fn": cls_key,
            "args": encoded, "nret": 0, "owner": self.addr, "name": cls_name,
            "resources": opts["resources"], "strategy": opts.get("strategy"),
            "actor_id": actor_id, "max_concurrency": opts.get("max_concurrency"),
            "concurrency_groups": opts.get("concurrency_groups"),
            "is_async": method_meta.get("__is_async__", False),
            "runtime_env": self._export_renv(opts.get("runtime_env")), "job": self.job_id,
            "method_meta": method_meta, "ns": self.namespace,
        }
        if _tracing.ENABLED:
            _tracing.inject(spec, "actor")
        self._inline_ready_args(spec)
        info = {
            "actor_id": actor_id, "name": opts.get("name"),
            "namespace": opts.get("namespace") or self.namespace,
            "lifetime": opts.get("lifetime"), "max_restarts": opts.get("max_restarts", 0),
            "owner": self.addr, "class_name": cls_name, "get_if_exists": opts.get("get_if_exists"),
            "max_task_retries": opts.get("max_task_retries", 0),
        }
        # args that are pending owned refs must be ready before the raylet runs __init__
        pend = [oid for oid, owner, inline in encoded[1] if owner == self.addr and inline is None]
        if pend:
            self.wait_refs(pend, len(pend), None)
            self._inline_ready_args(spec)
        existing = self.call_raylet("create_actor", info, {k: v for k, v in spec.items()
                                                            if not k.startswith("_")})
        with self.lock:
            ac = self.actors.get(actor_id)
            if ac is None:
                ac = self.actors[actor_id] = _ActorConn(actor_id)
            ac.max_task_retries = opts.get("max_task_retries", 0)
        self._holders_keepalive(actor_id, holders)
        self._subscribe_actor(actor_id)
        return existing

    def _holders_keepalive(self, actor_id, holders):
        if holders:
            if not hasattr(self, "_actor_arg_pins"):
                self._actor_arg_pins = {}
            self._actor_arg_pins[actor_id] = holders

    def _subscribe_actor(self, actor_id):
        with self.lock:
            ac = self.actors.get(actor_id)
            if ac is None:
                ac = self.actors[actor_id] = _ActorConn(actor_id)
            if ac.subscribed:
                return
            ac.subscribed = True
        self.call_async(self.raylet_addr, "subscribe_actor", (actor_id,),
                        lambda ok, v: self._on_actor_update(*v) if ok and v else None)

    def _on_actor_update(self, actor_id, state, addr, death, num_restarts=0):
        to_send = []
        to_fail = []
        with self.lock:
            ac = self.actors.get(actor_id)
            if ac is None:
                return
            if state == P.ALIVE:
                if ac.state == P.ALIVE and ac.addr == addr:
                    return
                ac.state, ac.addr = P.ALIVE, addr
                if ac.lost:  # restarted: tasks that died with the old process fail
                    lost, ac.lost = ac.lost, []
                    threading.Thread(target=self._fail_lost, args=(actor_id, lost, None),
                                     daemon=True).start()
                ac.num_restarts = num_restarts
                # resend in-flight (retryable) + queued, in sequence order
                pending = sorted(list(ac.inflight.values()) + list(ac.queue),
                                 key=lambda s: s["seq"])
                ac.inflight.clear()
                ac.queue.clear()
                for s in pending:
                    ac.inflight[s["tid"]] = s
                    to_send.append(s)
            elif state == P.DEAD:
                ac.state = P.DEAD
                ac.death = death
                to_fail = list(ac.inflight.values()) + list(ac.queue) + ac.lost
                ac.inflight.clear()
                ac.queue.clear()
                ac.lost = []
            else:
                if ac.state == P.ALIVE and state == P.RESTARTING:
                    self._requeue_inflight(ac)
                ac.state = state
        for s in to_send:
            self._send_actor_task(addr, s)
        for s in to_fail:
            self._fail_task(s, self._actor_error(actor_id, death))

    def _actor_error(self, actor_id, death):
        if isinstance(death, RayActorError):
            return death
        if isinstance(death, BaseException):
            e = ActorDiedError(actor_id.hex(), "The actor died because of an error raised in "
                               f"its creation task, {death}")
            e.cause = death
            return e
        return ActorDiedError(actor_id.hex(), death or "The actor died unexpectedly.")

    def _requeue_inflight(self, ac):
        # called with lock held; in-flight tasks either retry or fail
        fail = []
        for tid, s in list(ac.inflight.items()):
            if s.get("retries", 0) != 0:
                if s["retries"] > 0:
                    s["retries"] -= 1
                ac.queue.append(s)
            else:
                fail.append(s)
        ac.inflight.clear()
        if fail:
            ac.lost.extend(fail)

            def fallback(ac=ac, fail=fail):
                with self.lock:
                    left = [x for x in fail if x in ac.lost]
                    ac.lost = [x for x in ac.lost if x not in left]
                self._fail_lost(ac.actor_id, left, None)

            t = threading.Timer(5.0, fallback)
            t.daemon = True
            t.start()

    def _fail_lost(self, actor_id, specs, death):
        err = self._actor_error(actor_id, death) if death else \
            RayActorError(actor_id.hex(), "The actor died while running this task.")
        for sp in specs:
            self._fail_task(sp, err)

    def _on_actor_conn_lost(self, ac):
        with self.lock:
            if ac.state != P.ALIVE:
                return
            ac.state = P.RESTARTING
            self._requeue_inflight(ac)

    def submit_actor_task(self, actor_id, method, args, kwargs, opts):
        from ray_amd.object_ref import ObjectRef, ObjectRefGenerator

        tid = self.new_task_id()
        nret = opts.get("num_returns", 1)
        streaming = nret in ("streaming", "dynamic")
        encoded, holders = self._encode_args(args, kwargs)
        with self.lock:
            ac = self.actors.get(actor_id)
            if ac is None:
                ac = self.actors[actor_id] = _ActorConn(actor_id)
            limit = opts.get("max_pending_calls") or -1
            if limit > 0 and len(ac.inflight) + len(ac.queue) >= limit:
                from ray_amd.exceptions import PendingCallsLimitExceeded

                raise PendingCallsLimitExceeded(
                    f"The actor {actor_id.hex()} has {limit} pending calls from this caller "
                    f"(max_pending_calls={limit}); wait for some of them before submitting more")
            ac.seq += 1
            seq = ac.seq
        spec = {
            "tid": tid, "type": P.ACTOR_TASK, "actor_id": actor_id, "method": method,
            "args": encoded, "nret": -1 if streaming else nret, "owner": self.addr,
            "seq": seq, "name": opts.get("name") or method, "job": self.job_id,
            "retries": opts.get("max_task_retries", ac.max_task_retries),
            "concurrency_group": opts.get("concurrency_group"), "_holders": holders,
        }
        if opts.get("enable_task_events", True) is False:
            spec["no_events"] = True
        if _tracing.ENABLED:
            _tracing.inject(spec, "actor")
        with self.lock:
            if streaming:
                self.streams[tid] = _Stream()
            else:
                for i in range(nret):
                    self.owned[object_id_for_return(tid, i + 1)] = _Owned(tid)
            self.task_specs[tid] = spec
        self._note_child(tid)
        refs = [] if streaming else [ObjectRef(object_id_for_return(tid, i + 1), self.addr,
                                               _cw_obj=self) for i in range(nret)]
        if not spec.get("no_events"):
            self.task_events.append((tid, spec["name"], time.time(), None, None, actor_id,
                                     "SUBMITTED_TO_WORKER", P.ACTOR_TASK, self.job_id, 0, None))
        self._subscribe_actor(actor_id)
        # wait for owned pending args (ordering preserved: we block the caller)
        pend = [oid for oid, owner, inline in encoded[1] if owner == self.addr and inline is None]
        if pend:
            def go():
                self.wait_refs(pend, len(pend), None)
                self._inline_ready_args(spec)
                self._enqueue_actor_task(ac, spec)

            if threading.current_thread() is self.dispatcher:
                threading.Thread(target=go, daemon=True).start()
            else:
                go()
        else:
            self._enqueue_actor_task(ac, spec)
        if streaming:
            return ObjectRefGenerator(tid, self, self.addr)
        return refs

    def _enqueue_actor_task(self, ac, spec):
        send_to = None
        fail = None
        with self.lock:
            if ac.state == P.ALIVE:
                ac.inflight[spec["tid"]] = spec
                send_to = ac.addr
            elif ac.state == P.DEAD:
                fail = ac.death
            else:
                ac.queue.append(spec)
        if send_to:
            self._send_actor_task(send_to, spec)
        elif fail is not None or (ac.state == P.DEAD):
            self._fail_task(spec, self._actor_error(ac.actor_id, fail))

    def _send_actor_task(self, addr, spec):
        wire = {k: v for k, v in spec.items() if not k.startswith("_")}
        if not self.send(addr, (P.TASK, wire)):
            with self.lock:
                ac = self.actors.get(spec["actor_id"])
            if ac is not None:
                self._on_actor_conn_lost(ac)

    def _actor_call_finished(self, spec) -> bool:
        """Drop a finished (replied OR failed) actor call from its connection's books;
        True when that was the last call keeping a handle-less actor alive, i.e. the
        caller must now send ``actor_out_of_scope``."""
        with self.lock:
            ac = self.actors.get(spec["actor_id"])
            if ac is None:
                return False
            tid = spec["tid"]
            ac.inflight.pop(tid, None)
            if ac.queue:
                ac.queue = type(ac.queue)(s_ for s_ in ac.queue if s_["tid"] != tid)
            if ac.release_when_idle and not ac.inflight and not ac.queue and \
                    self.actor_handle_counts.get(ac.actor_id, 0) <= 0:
                ac.release_when_idle = False
                return True
        return False

    def _on_actor_task_reply(self, spec, returns, extra):
        release = self._actor_call_finished(spec)
        self._complete(spec, returns, extra, call_finished=True)
        if release and not self._stopped:
            self.notify_raylet("actor_out_of_scope", spec["actor_id"])

    def kill_actor(self, actor_id, no_restart=True):
        self.call_raylet("kill_actor", actor_id, no_restart)

    def actor_handle_created(self, actor_id):
        with self.lock:
            self.actor_handle_counts[actor_id] += 1

    def actor_handle_deleted(self, actor_id, owner_addr):
        kill = False
        with self.lock:
            self.actor_handle_counts[actor_id] -= 1
            if self.actor_handle_counts[actor_id] <= 0:
                del self.actor_handle_counts[actor_id]
                kill = (owner_addr == self.addr and actor_id not in self.actor_escaped)
                ac = self.actors.get(actor_id)
                if kill and ac is not None and (ac.inflight or ac.queue):
                    ac.release_when_idle = True  # after the submitted calls reply
                    kill = False
        if kill and not self._stopped:
            self.notify_raylet("actor_out_of_scope", actor_id)

    # ------------------------------------------------------------------ execution
    def _on_task(self, conn, msg):
        spec = msg[1]
        spec["_conn"] = conn
        if spec["type"] == P.ACTOR_TASK and self.actor_pools:
            self._dispatch_actor_task(spec)
        else:
            self.exec_queue.put(spec)

    def _take_queued(self, tid=None):
        """Remove unstarted normal tasks from the executor queue (one ``tid``, or all)."""
        q = self.exec_queue
        out = []
        with q.mutex:
            keep = collections.deque()
            for spec in q.queue:
                if spec is not None and spec["type"] == P.NORMAL_TASK and \
                        (tid is None or spec["tid"] == tid):
                    out.append(spec)
                else:
                    keep.append(spec)
            q.queue.clear()
            q.queue.extend(keep)
        return out

    def _requeue_to_owner(self, specs):
        for spec in specs:
            conn = spec.pop("_conn", None)
            self._send_reply(conn, spec["owner"], spec["tid"], [], {"requeue": True})

    def _on_steal(self, conn, msg):
        self._requeue_to_owner(self._take_queued(msg[1]))

    def _dispatch_actor_task(self, spec):
        if self.async_loop is not None:
            import asyncio

            asyncio.run_coroutine_threadsafe(self._run_async_actor_task(spec), self.async_loop)
            return
        grp = spec.get("concurrency_group")
        if grp is None:
            grp = self.actor_method_groups.get(spec["method"], "_default")
        pool = self.actor_pools.get(grp) or self.actor_pools["_default"]
        pool.submit(self._execute, spec)

    def run_task_loop(self):
        """Main-thread executor loop for worker processes."""
        prof_dir = os.environ.get("RAY_AMD_WORKER_CPROFILE")  # diagnostics (worker_main.py)
        prof, prof_t = None, time.monotonic()
        if prof_dir:
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        while not self.exiting:
            if prof is not None and time.monotonic() - prof_t > 2.0:
                prof_t = time.monotonic()
                prof.disable()
                prof.dump_stats(os.path.join(prof_dir, f"{self.mode}-{os.getpid()}-main.prof"))
                prof.enable()
            try:
                spec = self.exec_queue.get(timeout=1.0)
            except queue.Empty:
                continue
            if spec is None:
                break
            try:
                if spec["type"] == P.ACTOR_TASK and self.actor_pools:
                    self._dispatch_actor_task(spec)
                    continue
                self._execute(spec)
            except Exception:  # never let one task's bookkeeping end the worker loop
                traceback.print_exc()

    def _execute(self, spec):
        tid = spec["tid"]
        reply_to = spec["owner"] if spec["type"] != P.ACTOR_CREATION_TASK else None
        conn = spec.pop("_conn", None)
        if tid in self.cancelled:
            self._send_reply(conn, reply_to, tid, self._error_returns(
                spec, TaskCancelledError(tid.hex())), {})
            return
        self.current_task.tid = tid
        self.current_task.spec = spec
        self.current_task.ns = spec.get("ns")
        if spec["type"] == P.ACTOR_CREATION_TASK and spec.get("ns"):
            self._ns = spec["ns"]  # an actor lives in its creator's namespace
        self.current_task.lease_id = spec.get("lease_id")
        with self.lock:
            self.running[tid] = threading.get_ident()
        t0 = time.time()
        extra = {}
        name = spec.get("name") or "task"
        tspan = _tracing.on_execute_start(spec, spec.get("actor_id")) \
            if spec.get("trace") else None
        if not spec.get("no_events"):
            self.task_events.append((tid, name, t0, None, os.getpid(), spec.get("actor_id"),
                                     "RUNNING", spec["type"], spec.get("job"),
                                     spec.get("attempt", 0), None))
        try:
            if getattr(self, "setup_error", None):
                from ray_amd.exceptions import RuntimeEnvSetupError

                raise RuntimeEnvSetupError(self.setup_error)
            if spec["type"] == P.ACTOR_CREATION_TASK:
                returns = self._execute_actor_creation(spec)
            else:
                if spec["type"] == P.NORMAL_TASK:
                    fn = self._load_function(spec["fn"])
                elif spec["method"] == "__ray_terminate__":
                    raise _ActorExit()
                elif spec["method"] == "__ray_ready__":
                    fn = _ready
                elif spec["method"] == "__ray_call__":
                    inst = self.actor_instance
                    fn = lambda f, *a, **k: f(inst, *a, **k)  # noqa: E731
                else:
                    fn = getattr(self.actor_instance, spec["method"])
                args, kwargs = self._decode_args(spec["args"], spec["owner"])
                self._apply_runtime_env(spec)
                on_main = threading.current_thread() is threading.main_thread()
                if tid in self.cancelled:  # cancelled while its arguments were decoded
                    raise KeyboardInterrupt
                if on_main:
                    self._main_interruptible = True
                if spec["nret"] == -1:
                    returns = self._run_generator(spec, fn, args, kwargs, conn, reply_to)
                    extra["num_items"] = self._last_gen_count
                else:
                    result = fn(*args, **kwargs)
                    if on_main:
                        self._main_interruptible = False
                    if spec.get("dynamic"):
                        result = _DynamicRefs([self.put_object(v) for v in result])
                    returns = self._package_returns(spec, result)
                if spec.get("max_calls") and spec["type"] == P.NORMAL_TASK:
                    extra["worker_exit"] = self._count_call(spec)
        except _ActorExit:
            returns = self._package_returns(spec, None) if spec["nret"] != -1 else []
            self._send_reply(conn, reply_to, tid, returns, extra)
            self._exit_actor()
            return
        except KeyboardInterrupt:
            returns = self._error_returns(spec, TaskCancelledError(tid.hex()))
        except BaseException as e:  # noqa: BLE001
            err = RayTaskError.from_exception(e, name, pid=os.getpid(),
                                              actor_repr=repr(self.actor_instance)
                                              if self.actor_instance is not None else None)
            if spec["type"] == P.ACTOR_CREATION_TASK:
                returns = [("__init_error__", ser.serialize_error(err).to_bytes())]
            else:
                returns = self._error_returns(spec, err)
                extra["app_error"] = True
                extra["exc_type"] = type(e).__name__
        finally:
            if threading.current_thread() is threading.main_thread():
                self._main_interruptible = False
            with self.lock:
                self.running.pop(tid, None)
                self._children.pop(tid, None)
            self.current_task.tid = None
            self.current_task.spec = None
            if tspan is not None:
                _tracing.on_execute_end(tspan, bool(extra.get("app_error")))
        if not spec.get("no_events"):
            self.task_events.append((tid, name, t0, time.time(), os.getpid(),
                                     spec.get("actor_id"), "FAILED" if extra.get("app_error")
                                     else "FINISHED", spec["type"], spec.get("job"),
                                     spec.get("attempt", 0), extra.get("exc_type")))
        self._send_reply(conn, reply_to, tid, returns, extra)

    def _count_call(self, spec):
        """max_calls: True once this worker has run the function max_calls times; the
        owner then returns the lease with worker_dead=True, so the raylet retires this
        process and the next call gets a fresh worker (reference: remote_function.py
        max_calls; the worker exits after that many invocations)."""
        calls = self.__dict__.setdefault("_fn_calls", {})
        k = repr(spec["fn"])
        calls[k] = calls.get(k, 0) + 1
        return calls[k] >= spec["max_calls"]

    # ---------------------------------------------------------------- setup hooks
    _HOOK_NS = b"__runtime_env__"

    def _export_renv(self, renv):
        """A callable ``worker_process_setup_hook`` travels as ``kv:<key>``: pickled once
        into the internal KV, fetched by each worker process that starts with this env
        (reference: _private/runtime_env/setup_hook.py)."""
        if not renv or not isinstance(renv, dict):
            return renv
        hook = renv.get("worker_process_setup_hook")
        if hook is None or isinstance(hook, str):
            return renv
        if not callable(hook):
            raise TypeError("worker_process_setup_hook must be a callable or an import path "
                            f"string, got {type(hook).__name__}")
        import hashlib

        import cloudpickle

        blob = cloudpickle.dumps(hook)
        key = "setup_hook:" + hashlib.sha1(blob).hexdigest()
        exported = self.__dict__.setdefault("_exported_hooks", set())
        if key not in exported:
            self.call_raylet("kv_put", self._HOOK_NS, key.encode(), blob, True)
            exported.add(key)
        out = dict(renv)
        out["worker_process_setup_hook"] = "kv:" + key
        return out

    def run_setup_hook(self, hook: str):
        """Run once at worker start; a failure fails every task this worker runs with
        RuntimeEnvSetupError."""
        import traceback

        try:
            if hook.startswith("kv:"):
                import cloudpickle

                blob = self.call_raylet("kv_get", self._HOOK_NS, hook[3:].encode())
                if blob is None:
                    raise RuntimeError(f"setup hook {hook[3:]} not found in the internal KV")
                fn = cloudpickle.loads(blob)
            else:
                import importlib

                mod, _, attr = hook.rpartition(".")
                fn = getattr(importlib.import_module(mod), attr)
            fn()
        except BaseException:  # noqa: BLE001
            self.setup_error = ("worker_process_setup_hook failed:\n" +
                                traceback.format_exc())

    def _apply_runtime_env(self, spec):
        renv = spec.get("runtime_env")
        if renv and renv.get("env_vars"):
            os.environ.update({k: str(v) for k, v in renv["env_vars"].items()})

    def _send_reply(self, conn, reply_to, tid, returns, extra):
        if any(r[1] == P.RET_STORE for r in returns):
            extra["node"] = self.node_hex
        evs = None
        if reply_to is not None and self.task_events:
            # this worker's task events ride on the reply; the owner forwards them with its
            # own batch (one raylet message per owner flush instead of one per task)
            q = self.task_events
            evs = _drain(q)
            if evs:
                extra["events"] = evs
        msg = (P.TASK_REPLY, tid, returns, extra)
        if reply_to is not None and self.send(reply_to, msg):
            return
        if evs:
            self.task_events.extend(evs)
            extra.pop("events", None)
        if conn is not None:
            self.io.send(conn, _dumps(msg))

    def _error_returns(self, spec, exc):
        data = ser.serialize_error(exc).to_bytes()
        n = spec["nret"] if spec["nret"] > 0 else 0
        if spec["nret"] == -1:
            return [(object_id_for_return(spec["tid"], 0x7FFFFFFF), P.RET_INLINE, data, None)]
        return [(object_id_for_return(spec["tid"], i + 1), P.RET_INLINE, data, None)
                for i in range(n)]

    def _package_one(self, oid, value, owner):
        sobj = ser.serialize(value, oid)
        contained = None
        if sobj.refs:
            contained = []
            for r in sobj.refs:
                contained.append((r._id, r._owner))
                self._pin_for(r, owner)
        if sobj.total <= INLINE_MAX and not sobj.gpu:
            return (oid, P.RET_INLINE, sobj.to_bytes(), contained)
        self.store.put_serialized(oid, sobj, pinned=True)
        return (oid, P.RET_STORE, sobj.total, contained)

    def _pin_for(self, ref, owner_addr):
        """Register `owner_addr` as a borrower of `ref` before handing it over."""
        if ref._owner == self.addr:
            with self.lock:
                o = self.owned.get(ref._id)
                if o is not None:
                    if o.borrowers is None:
                        o.borrowers = {}
                    o.borrowers[owner_addr] = o.borrowers.get(owner_addr, 0) + 1
        elif ref._owner != owner_addr:
            try:
                self.call(ref._owner, "add_borrower", ref._id, owner_addr, timeout=30)
            except Exception:
                pass

    def _package_returns(self, spec, result):
        n = spec["nret"]
        tid = spec["tid"]
        owner = spec["owner"]
        if n == 0:
            return []
        if n == 1:
            return [self._package_one(object_id_for_return(tid, 1), result, owner)]
        if not isinstance(result, (tuple, list)) or len(result) != n:
            raise ValueError(f"Task returned {result!r} but num_returns={n}")
        return [self._package_one(object_id_for_return(tid, i + 1), v, owner)
                for i, v in enumerate(result)]

    def _on_stream_ack(self, conn, msg):
        tid, consumed = msg[1], msg[2]
        cv = self._gen_ack_cv()
        with cv:
            if consumed > self._gen_acks.get(tid, 0):
                self._gen_acks[tid] = consumed
                cv.notify_all()

    def _gen_ack_cv(self):
        cv = getattr(self, "_gacv", None)
        if cv is None:
            self._gen_acks = {}
            self._gacv = cv = threading.Condition()
        return cv

    def _gen_throttle(self, spec, produced):
        """_generator_backpressure_num_objects: block the generator while ``produced`` -
        consumed >= the threshold (the owner acks every item its caller takes)."""
        bp = spec.get("gen_bp", 0)
        if not bp:
            return
        tid = spec["tid"]
        cv = self._gen_ack_cv()
        with cv:
            while produced - self._gen_acks.get(tid, 0) >= bp and not self._stopped:
                cv.wait(0.5)

    def _run_generator(self, spec, fn, args, kwargs, conn, reply_to):
        tid = spec["tid"]
        owner = spec["owner"]
        gen = fn(*args, **kwargs)
        i = 0
        if hasattr(gen, "__anext__"):
            import asyncio

            loop = asyncio.new_event_loop()
            try:
                while True:
                    try:
                        v = loop.run_until_complete(gen.__anext__())
                    except StopAsyncIteration:
                        break
                    ret = self._package_one(object_id_for_return(tid, i + 1), v, owner)
                    self.send(owner, (P.STREAM_ITEM, tid, i, ret, self.node_hex))
                    i += 1
                    self._gen_throttle(spec, i)
            finally:
                loop.close()
        else:
            for v in gen:
                ret = self._package_one(object_id_for_return(tid, i + 1), v, owner)
                self.send(owner, (P.STREAM_ITEM, tid, i, ret, self.node_hex))
                i += 1
                self._gen_throttle(spec, i)
        self._last_gen_count = i
        if spec.get("gen_bp"):
            with self._gen_ack_cv():
                self._gen_acks.pop(tid, None)
        return []

    # ---- actor side
    def _execute_actor_creation(self, spec):
        cls = self._load_function(spec["fn"])
        args, kwargs = self._decode_args(spec["args"], spec["owner"])
        self._apply_runtime_env(spec)
        self.actor_id = spec["actor_id"]
        self.actor_spec = spec
        self.current_task.actor_id = self.actor_id
        meta = spec.get("method_meta") or {}
        is_async = spec.get("is_async")
        groups = spec.get("concurrency_groups") or {}
        self.actor_method_groups = meta.get("__groups__", {})
        instance = cls.__new__(cls)
        self.actor_instance = instance
        if is_async:
            import asyncio

            loop = asyncio.new_event_loop()
            self.async_loop = loop
            self._async_sem = asyncio.Semaphore(spec.get("max_concurrency") or 1000)
            t = threading.Thread(target=loop.run_forever, name="ray_amd-asyncio", daemon=True)
            t.start()
            fut = asyncio.run_coroutine_threadsafe(self._async_init(instance, args, kwargs), loop)
            fut.result()
        else:
            instance.__init__(*args, **kwargs)
        mc = spec.get("max_concurrency") or 1
        if not is_async and (mc > 1 or groups):
            from concurrent.futures import ThreadPoolExecutor

            self.actor_pools["_default"] = ThreadPoolExecutor(mc, "ray_amd-actor")
            for g, n in groups.items():
                self.actor_pools[g] = ThreadPoolExecutor(n, f"ray_amd-cg-{g}")
        elif is_async:
            self.actor_pools["_default"] = None
        return []

    async def _async_init(self, instance, args, kwargs):
        instance.__init__(*args, **kwargs)

    async def _run_async_actor_task(self, spec):
        import asyncio
        import inspect

        tid = spec["tid"]
        conn = spec.pop("_conn", None)
        owner = spec["owner"]
        me = asyncio.current_task()
        with self.lock:
            self._async_tasks[tid] = (asyncio.get_running_loop(), me)
        try:
            await self._run_async_actor_task_body(spec, tid, conn, owner)
        except asyncio.CancelledError:
            self._send_reply(conn, owner, tid,
                             self._error_returns(spec, TaskCancelledError(tid.hex())), {})
        finally:
            with self.lock:
                self._async_tasks.pop(tid, None)

    async def _run_async_actor_task_body(self, spec, tid, conn, owner):
        import asyncio
        import inspect

        if tid in self.cancelled:
            raise asyncio.CancelledError()
        async with self._async_sem:
            self.current_task.tid = tid
            try:
                m = spec["method"]
                if m == "__ray_terminate__":
                    raise _ActorExit()
                if m == "__ray_ready__":
                    fn = _ready
                elif m == "__ray_call__":
                    inst = self.actor_instance
                    fn = lambda f, *a, **k: f(inst, *a, **k)  # noqa: E731
                else:
                    fn = getattr(self.actor_instance, m)
                loop = asyncio.get_running_loop()
                enc = spec["args"]
                if all(inl is not None for _, _, inl in (enc[1] or ())):
                    # every argument is inline: decoding cannot block, skip the thread hop
                    args, kwargs = self._decode_args(enc, owner)
                else:  # may wait for ObjectRef arguments: off the event loop
                    args, kwargs = await loop.run_in_executor(None, self._decode_args, enc, owner)
                if spec["nret"] == -1 and inspect.isasyncgenfunction(
                        getattr(fn, "__func__", fn)):
                    # async generators run on the actor's own event loop (they may share
                    # loop-bound state with the actor's other coroutines)
                    gen = fn(*args, **kwargs)
                    i = 0
                    async for v in gen:
                        ret = self._package_one(object_id_for_return(tid, i + 1), v, owner)
                        self.send(owner, (P.STREAM_ITEM, tid, i, ret, self.node_hex))
                        i += 1
                    returns = []
                    extra = {"num_items": i}
                elif spec["nret"] == -1:
                    returns = await loop.run_in_executor(None, self._run_generator_async_bridge,
                                                         spec, fn, args, kwargs)
                    extra = {"num_items": self._last_gen_count}
                else:
                    r = fn(*args, **kwargs)
                    if inspect.isawaitable(r):
                        r = await r
                    if _small_value(r):  # serialising a scalar / short bytes is cheap
                        returns = self._package_returns(spec, r)
                    else:  # large values are written to the object store off the loop
                        returns = await loop.run_in_executor(None, self._package_returns, spec,
                                                             r)
                    extra = {}
            except _ActorExit:
                self._send_reply(conn, owner, tid, self._package_returns(spec, None), {})
                self._exit_actor()
                return
            except asyncio.CancelledError:
                raise
            except BaseException as e:  # noqa: BLE001
                err = RayTaskError.from_exception(e, spec.get("name", "task"), pid=os.getpid())
                returns = self._error_returns(spec, err)
                extra = {"app_error": True, "exc_type": type(e).__name__}
        self._send_reply(conn, owner, tid, returns, extra)

    def _run_generator_async_bridge(self, spec, fn, args, kwargs):
        return self._run_generator(spec, fn, args, kwargs, None, spec["owner"])

    def _exit_actor(self):
        self.exiting = True
        self.notify_raylet("actor_exit", self.actor_id)
        time.sleep(0.05)
        os._exit(0)

    def _flush_task_events(self):
        self._events_flushed = time.monotonic()
        q = self.task_events
        ev = _drain(q)
        if ev:
            self.notify_raylet("task_events", ev)

    # ------------------------------------------------------------------ local mode
    def _run_local(self, spec):
        fn = self.fn_cache[spec["fn"]]
        args, kwargs = self._decode_args(spec["args"], self.addr)
        try:
            r = fn(*args, **kwargs)
            returns = self._package_returns(spec, r)
        except BaseException as e:  # noqa: BLE001
            returns = self._error_returns(spec, RayTaskError.from_exception(
                e, spec.get("name", "task"), pid=os.getpid()))
        self._complete(spec, returns, {})

    # ------------------------------------------------------------------ shutdown
    def shutdown(self):
        if self._stopped:
            return
        self._stopped = True
        try:
            self._flush_task_events()
        except Exception:
            pass
        try:
            self.io.stop()
        except Exception:
            pass
        # the dispatcher may still be inside io.poll(): let it leave the native loop before the
        # interpreter can finalize (and free the IOLoop) under it
        d = getattr(self, "dispatcher", None)
        if d is not None and d is not threading.current_thread():
            d.join(timeout=2.0)
        try:
            os.unlink(self.addr)
        except OSError:
            pass


class _ArgRef:
    __slots__ = ("i",)

    def __init__(self, i):
        self.i = i

    def __reduce__(self):
        return (_ArgRef, (self.i,))


class _ActorExit(BaseException):
    pass


class _DynamicRefs(list):
    """Value of a num_returns="dynamic" task: iterable of ObjectRefs."""


def _ready():
    return True


def _small_value(v) -> bool:
    """Return values packaged inline on an async actor's event loop."""
    if v is None or isinstance(v, (bool, int, float)):
        return True
    return isinstance(v, (bytes, str)) and len(v) <= 4096
