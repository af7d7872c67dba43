"""Raylet + GCS process for a ray_amd node (reference: src/ray/raylet/node_manager.cc,
worker_pool.cc, local_task_manager.cc; src/ray/gcs/gcs_server/{gcs_actor_manager,
gcs_placement_group_manager,gcs_kv_manager,gcs_job_manager}.cc).

One single-threaded event loop over the native IOLoop. Scheduling decisions
(resource fit, GPU instance assignment, hybrid/spread/affinity policies,
placement-group bundle placement) are delegated to the native
``_core.Scheduler``; this module owns the worker pool, leases, the actor
lifecycle (create → ALIVE → RESTARTING → DEAD), named actors, placement groups,
the internal KV, jobs and task events.
"""

from __future__ import annotations

import argparse
import collections
import json
import os
import signal
import subprocess
import sys
import threading
import time
import traceback

from ray_amd._native import _core

from . import protocol as P
from . import serialization as ser
from . import shm_segment
from .object_store import start_prefault, table_capacity

_dumps = P.dumps


class WorkerRec:
    __slots__ = ("wid", "pid", "addr", "conn", "key", "state", "lease", "proc", "token",
                 "actor_id", "job", "gpu_ids", "mode", "idle_since", "namespace", "started",
                 "node", "death_cause")

    def __init__(self):
        self.wid = None
        self.pid = None
        self.addr = None
        self.conn = None
        self.key = None
        self.state = "starting"
        self.lease = None
        self.proc = None
        self.token = None
        self.actor_id = None
        self.job = None
        self.gpu_ids = ()
        self.mode = "worker"
        self.idle_since = time.monotonic()
        self.namespace = None
        self.started = time.monotonic()
        self.node = None


class Lease:
    __slots__ = ("lid", "worker", "alloc", "resources", "owner", "strategy", "cpu_released",
                 "pg", "actor_id", "retriable", "granted_at")

    def __init__(self, lid, worker, alloc, resources, owner, strategy, retriable=True):
        self.lid = lid
        self.worker = worker
        self.alloc = alloc
        self.resources = resources
        self.owner = owner
        self.strategy = strategy
        self.cpu_released = False
        self.pg = None
        self.actor_id = None
        self.retriable = retriable
        self.granted_at = time.monotonic()


def select_worker_to_kill(leases, policy: str = "group_by_owner"):
    """Memory-pressure victim (reference: src/ray/raylet/worker_killing_policy_*.cc).

    group_by_owner: group running leases by owner; prefer retriable groups, then the
    largest group, then the newest; inside the group kill the NEWEST lease (the work
    least far along). retriable_fifo: retriable first, then the OLDEST lease.
    Returns (lease, should_retry) or (None, False)."""
    if not leases:
        return None, False
    if policy == "retriable_fifo":
        best = sorted(leases, key=lambda l: (0 if l.retriable else 1, l.granted_at))[0]
        return best, best.retriable
    groups = {}
    for l in leases:
        key = (l.owner, True) if l.retriable else ("__non_retriable__", False)
        groups.setdefault(key, []).append(l)
    ordered = sorted(groups.items(), key=lambda kv: (0 if kv[0][1] else 1, -len(kv[1]),
                                                     -max(x.granted_at for x in kv[1])))
    (_, retriable), members = ordered[0]
    victim = max(members, key=lambda x: x.granted_at)
    return victim, retriable and len(members) > 1


class LeaseReq:
    __slots__ = ("rid", "conn", "req", "alloc", "node", "waiting_token", "cb", "t0", "warned",
                 "resources", "shape")

    def __init__(self, rid, conn, req, cb=None):
        self.rid = rid
        self.conn = conn
        self.req = req
        self.alloc = None
        self.node = None
        self.waiting_token = None
        self.cb = cb
        self.t0 = time.monotonic()
        self.warned = False
        self.resources = None
        self.shape = None  # (resources, strategy, target, hard labels, soft labels), resolved once


class ActorRec:
    def __init__(self, info, spec):
        self.info = info
        self.spec = spec
        self.aid = info["actor_id"]
        self.state = P.PENDING_CREATION
        self.worker = None
        self.lease = None
        self.death = None
        self.restarts = 0
        self.max_restarts = info.get("max_restarts") or 0
        self.no_restart = False
        self.subscribers = set()
        self.pid = None
        self.start_time = time.time()
        self.end_time = None


class PGRec:
    def __init__(self, pg_id, bundles, strategy, name, lifetime, owner, namespace):
        self.pg_id = pg_id
        self.bundles = bundles
        self.strategy = strategy
        self.name = name
        self.lifetime = lifetime
        self.owner = owner
        self.namespace = namespace
        self.state = "PENDING"
        self.nodes = []
        self.waiters = []
        self.created_at = time.time()


_PG_STRATEGY = {"PACK": 0, "SPREAD": 1, "STRICT_PACK": 2, "STRICT_SPREAD": 3}


def detect_cpus() -> int:
    """Usable CPUs: affinity mask, capped by a cgroup CPU quota (reference:
    ray._private.utils.get_num_cpus, which also honours container quotas)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:  # cgroup v2: "<quota|max> <period>"
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, max(1, int(quota)))
    return max(1, n)


def node_resources(args, node_ip, head):
    """Resource vector a node advertises (reference: resource_spec.py auto-detection)."""
    res = json.loads(args.resources or "{}")
    ncpu = args.num_cpus if args.num_cpus is not None else detect_cpus()
    ngpu = args.num_gpus if args.num_gpus is not None else detect_gpus()
    total = {"CPU": float(ncpu), "memory": float(args.memory or 8 << 30),
             "object_store_memory": float(args.object_store_memory),
             f"node:{node_ip}": 1.0}
    if ngpu:
        total["GPU"] = float(ngpu)
        from ray_amd.util.accelerators import detect_accelerator_type

        acc = os.environ.get("RAY_AMD_ACCELERATOR_TYPE") or detect_accelerator_type()
        if acc:  # reference: accelerator_type:<type> node resource (amd_gpu.py)
            total[f"accelerator_type:{acc}"] = 1.0
    if head:
        total["node:__internal_head__"] = 1.0
    total.update({k: float(v) for k, v in res.items()})
    return total, ncpu


def detect_gpus() -> int:
    """Count AMD GPUs without initialising HIP (reads KFD topology)."""
    env = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") \
        or os.environ.get("CUDA_VISIBLE_DEVICES")
    if env is not None and env.strip() != "":
        return len([x for x in env.split(",") if x.strip() != ""])
    n = 0
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for d in os.listdir(base):
            try:
                with open(os.path.join(base, d, "properties")) as f:
                    props = f.read()
                for line in props.splitlines():
                    if line.startswith("simd_count") and int(line.split()[1]) > 0:
                        n += 1
                        break
            except OSError:
                continue
    except OSError:
        return 0
    return n


class Raylet:
    def __init__(self, args):
        self.session_dir = args.session_dir
        os.makedirs(os.path.join(self.session_dir, "sockets"), exist_ok=True)
        os.makedirs(os.path.join(self.session_dir, "logs"), exist_ok=True)
        self.addr = os.path.join(self.session_dir, "sockets", "raylet.sock")
        self.node_id = _core.random_id(16)
        from ray_amd._private.reporter import NodeReporter

        # node / MI355X telemetry (reporter_agent.py parity); remote nodes push theirs
        self.reporter = NodeReporter(self.node_id.hex(), self.session_dir).start()
        self.node_stats = {}  # node hex -> latest sample pushed by that node's agent
        self.node_ip = os.environ.get("RAY_AMD_NODE_IP", "127.0.0.1")
        # anonymous memfd segment: freed by the kernel with the last process holding it,
        # however this raylet exits (shm_segment.py; plasma's unlink-after-map model)
        self.store_path, self._store_fd = shm_segment.create(args.store_path)
        self.spill_dir = os.path.join(self.session_dir, "spill")
        os.makedirs(self.spill_dir, exist_ok=True)
        self.store = _core.ShmStore(self.store_path, args.object_store_memory, True,
                                    table_capacity(args.object_store_memory))
        start_prefault(self.store, args.object_store_memory)
        from .object_store import SpillManager

        self.spiller = SpillManager(self.store, self.spill_dir).start()
        self.io = _core.IOLoop()
        self.io.listen_unix(self.addr)
        self.sched = _core.Scheduler()
        total, ncpu = node_resources(args, self.node_ip, head=True)
        self.labels = json.loads(args.labels or "{}")
        self.labels.setdefault("ray.io/node_id", self.node_id.hex())
        for k in total:
            if k.startswith("accelerator_type:"):  # label twin of the resource
                self.labels.setdefault("ray.io/accelerator-type", k.split(":", 1)[1])
        self.sched.add_node(self.node_id.hex(), total, self.labels)
        self.total = total
        self.num_cpus = ncpu
        # cluster membership (reference: gcs_node_manager.cc). The head raylet schedules
        # the whole cluster; worker-node agents (node_agent.py) spawn workers and serve
        # their node's object store.
        self.node_hex = self.node_id.hex()
        self.node_recs = {self.node_hex: {
            "node_id": self.node_hex, "addr": self.addr, "conn": None,
            "store_path": self.store_path, "spill_dir": self.spill_dir, "labels": self.labels,
            "resources": total, "alive": True, "pid": os.getpid(), "is_head": True,
            "start_time": time.time(), "num_cpus": ncpu}}
        self.node_conn = {}
        self.conn_addr = {}
        self.addr_conn = {}
        self.conn_worker = {}
        self.workers = {}  # wid -> WorkerRec
        self.starting = {}  # token -> WorkerRec
        self.idle = collections.defaultdict(list)
        self.leases = {}
        self.pending = collections.deque()
        self.kv = {}
        self.actors = {}
        self.named = {}
        self.pgs = {}
        self.pg_names = {}
        self.jobs = {}
        self.job_counter = 0
        self.task_events = collections.deque(maxlen=100000)  # terminal events (timeline)
        self.task_table: "collections.OrderedDict[bytes, dict]" = collections.OrderedDict()
        self.app_metrics: dict = {}  # pid -> metric snapshots (ray_amd.util.metrics)
        self.next_token = 1
        self.next_lease = 1
        self.dirty = True
        self.stop = False
        self.max_starting = max(4, ncpu)
        self.python = sys.executable
        self.internal_cb = {}
        self.next_internal = -1
        self.start_time = time.time()
        self.gpu_arenas = {}
        # GCS durability (reference: gcs_server + gcs_table_storage on an external store):
        # with RAY_AMD_GCS_STORAGE_PATH set, the head persists KV, jobs, detached actors and
        # detached placement groups to <path>/gcs_snapshot.pkl and a restarted head reloads
        # them (detached actors are re-created, counting one restart)
        self._gcs_path = os.environ.get("RAY_AMD_GCS_STORAGE_PATH") if args.head else None
        self._gcs_dirty = False
        self._gcs_saved = 0.0
        self._gcs_writer = None
        self.gcs_restored = None
        # detached actors of the previous head that lived on OTHER nodes: their workers may
        # survive the head restart and re-attach (rpc_reattach_actor) within the grace
        # period; the ones that do not are re-created from their specs afterwards
        self._readopt: dict = {}
        self._readopt_grace = float(os.environ.get("RAY_AMD_GCS_READOPT_S", "5"))
        if self._gcs_path:
            os.makedirs(self._gcs_path, exist_ok=True)
            self._gcs_restore()
        # memory monitor + worker killing policy (reference: memory_monitor.cc,
        # worker_killing_policy.cc; config names follow RAY_memory_usage_threshold etc.)
        env = os.environ
        self.mem_refresh = float(env.get("RAY_memory_monitor_refresh_ms", "250")) / 1000.0
        self.mem_monitor = _core.MemoryMonitor(
            float(env.get("RAY_memory_usage_threshold", "0.95")),
            int(env.get("RAY_min_memory_free_bytes", "-1")),
            env.get("RAY_AMD_CGROUP_ROOT", "/sys/fs/cgroup"), "/proc") \
            if self.mem_refresh > 0 else None
        self.kill_policy = env.get("RAY_worker_killing_policy", "group_by_owner")
        self._mem_last = 0.0
        self._oom_victim = None  # (worker rec, deadline) of the last kill, until it exits
        self.death_causes: "collections.OrderedDict[str, str]" = collections.OrderedDict()
        self.oom_kills = 0

    # ------------------------------------------------------------------ io helpers
    def send(self, conn, msg):
        self.io.send(conn, _dumps(msg))

    def reply(self, conn, rid, ok, value):
        if rid and conn is not None:
            self.send(conn, (P.RESP, rid, ok, value))

    def run(self):
        handlers = {P.REQ: self.on_req, P.HELLO: self.on_hello, P.TASK_REPLY: self.on_task_reply,
                    P.RESP: self.on_resp}
        last_tick = 0.0
        prof_dir = os.environ.get("RAY_AMD_WORKER_CPROFILE")  # diagnostics (worker_main.py)
        prof, prof_t = None, 0.0
        if prof_dir:
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        while not self.stop:
            if prof is not None and time.monotonic() - prof_t > 2.0:
                prof_t = time.monotonic()
                prof.disable()
                prof.dump_stats(os.path.join(prof_dir, f"raylet-{os.getpid()}.prof"))
                prof.enable()
            ev = self.io.poll(20, 4096)
            for typ, conn, payload in ev:
                try:
                    if typ == 0:
                        msg = P.loads(payload)
                        h = handlers.get(msg[0])
                        if h:
                            h(conn, msg)
                    elif typ == 2:
                        self.on_closed(conn)
                except Exception:
                    traceback.print_exc()
            now = time.monotonic()
            if self.dirty or now - last_tick > 0.1:
                self.dirty = False
                try:
                    self.try_schedule()
                    if now - last_tick > 0.1:
                        last_tick = now
                        self.tick()
                except Exception:
                    traceback.print_exc()
        self.shutdown()

    def on_hello(self, conn, msg):
        self.conn_addr[conn] = msg[1]
        self.addr_conn[msg[1]] = conn

    def on_resp(self, conn, msg):
        pass

    def on_req(self, conn, msg):
        _, rid, method, args = msg
        h = getattr(self, "rpc_" + method, None)
        if h is None:
            self.reply(conn, rid, False, f"unknown raylet method {method}")
            return
        try:
            h(conn, rid, *args)
        except Exception as e:  # noqa: BLE001
            traceback.print_exc()
            self.reply(conn, rid, False, e if _picklable(e) else RuntimeError(repr(e)))

    # ------------------------------------------------------------------ registration
    def rpc_register(self, conn, rid, mode, wid, pid, addr, job_id, namespace, token,
                     node_hex=None):
        w = None
        if mode == "worker":
            w = self.starting.pop(token, None)
        if w is None:
            w = WorkerRec()
            rec = self.node_recs.get(node_hex or "")
            w.node = node_hex if rec is not None and rec["alive"] else self.node_hex
        w.wid, w.pid, w.addr, w.conn, w.mode = wid, pid, addr, conn, mode
        self.conn_worker[conn] = w
        self.workers[wid] = w
        if mode == "driver":
            self.job_counter += 1
            job_id = self.job_counter
            w.state = "driver"
            w.job = job_id
            w.namespace = namespace or f"anon-{job_id}"
            self._gcs_dirty = True
            self.jobs[job_id] = {"job_id": job_id, "driver_pid": pid, "driver_addr": addr,
                                 "start_time": time.time(), "end_time": None,
                                 "status": "RUNNING", "namespace": w.namespace,
                                 "sys_path": None}
        else:
            w.state = "idle"
            w.idle_since = time.monotonic()
            if w.key is not None:
                self.idle[w.key].append(w)
            self.dirty = True
        nrec = self.node_recs[w.node]
        info = {"node_id": bytes.fromhex(w.node),
                "job_id": w.job if mode == "driver" else job_id,
                "namespace": w.namespace if mode == "driver" else namespace,
                "store_path": nrec["store_path"], "spill_dir": nrec["spill_dir"],
                "node_ip": self.node_ip, "session_dir": self.session_dir,
                "resources": nrec["resources"], "head_node_id": self.node_hex}
        self.reply(conn, rid, True, info)

    def rpc_set_job_info(self, conn, rid, job_id, sys_path, runtime_env, job_config=None):
        j = self.jobs.get(job_id)
        if j is not None:
            j["sys_path"] = sys_path
            j["runtime_env"] = runtime_env
            if job_config is not None:
                j["metadata"] = dict(job_config.get("metadata") or {})
                j["job_config"] = job_config
        self.reply(conn, rid, True, None)

    # ------------------------------------------------------------------ worker pool
    def _pool_key(self, job, renv, gpu_ids, node, visible=()):
        # `visible`: GPUs the worker process sees (HIP_VISIBLE_DEVICES) when it differs from
        # its own assignment — a Train worker group shares the union of its placement
        # group's GPUs on the node so RCCL ranks see their xGMI peers, exactly like
        # torchrun. Decided HERE, before the process exists, so HIP initialises with it.
        return (job, json.dumps(renv, sort_keys=True, default=str) if renv else None,
                tuple(gpu_ids) if gpu_ids else (), node, tuple(visible))

    def _shared_visible(self, lr, gpu_ids):
        st = lr.req.get("strategy")
        if not gpu_ids or not isinstance(st, dict) or st.get("type") != "pg" or \
                not st.get("share_gpus"):
            return ()
        pg = self.pgs.get(st["pg_id"])
        if pg is None or not pg.nodes:
            return ()
        inst = self.sched.pg_gpu_instances(st["pg_id"])
        ids = set(gpu_ids)
        for b, node in enumerate(pg.nodes):
            if node == lr.node and b < len(inst):
                ids.update(inst[b])
        return tuple(sorted(ids))

    def _start_worker(self, key, renv, job):
        w = WorkerRec()
        w.token = self.next_token
        self.next_token += 1
        w.key = key
        w.job = job
        w.gpu_ids = key[2]
        w.node = node = key[3]
        env = dict(os.environ)
        env["RAY_AMD_NODE_ID"] = node
        j = self.jobs.get(job) or {}
        if j.get("sys_path"):
            env["RAY_AMD_JOB_SYS_PATH"] = json.dumps(j["sys_path"])
        pp = env.get("PYTHONPATH", "")
        pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = pkg_root + (os.pathsep + pp if pp else "")
        if w.gpu_ids:
            vis = os.environ.get("HIP_VISIBLE_DEVICES")
            shown = key[4] if len(key) > 4 and key[4] else w.gpu_ids
            ids = [str(i) for i in shown]
            if vis:
                base = [x for x in vis.split(",") if x.strip() != ""]
                ids = [base[i] for i in shown if i < len(base)]
            env["HIP_VISIBLE_DEVICES"] = ",".join(ids)
            env.pop("CUDA_VISIBLE_DEVICES", None)
            env.pop("ROCR_VISIBLE_DEVICES", None)
            env["RAY_AMD_GPU_IDS"] = ",".join(str(i) for i in w.gpu_ids)
            # device ordinal of this worker's (first) GPU inside its visible set
            env["RAY_AMD_LOCAL_DEVICE"] = str(list(shown).index(w.gpu_ids[0]))
        if os.environ.get("RAY_AMD_WORKER_MALLOC_TUNING", "1") == "1":
            # large temporaries (decoded image blocks, rollout arrays) are recycled from
            # the worker's heap instead of a fresh mmap per allocation: a fresh 36 MiB
            # mapping costs ~9k page faults, more than the work that fills it (measured:
            # the data bench's read task 35 -> 13 ms). Arrays above 64 MiB are still mapped
            # and unmapped on free, and more than 256 MiB free at the heap top is returned,
            # so a worker's RSS (what the memory monitor watches) stays near its live set.
            env.setdefault("MALLOC_MMAP_THRESHOLD_", str(64 << 20))
            env.setdefault("MALLOC_TRIM_THRESHOLD_", str(256 << 20))
        allr = {}
        for src in (j.get("runtime_env") or {}, renv or {}):
            allr.update(src)
        for k, v in (allr.get("env_vars") or {}).items():
            env[k] = str(v)
        if allr.get("worker_process_setup_hook"):
            env["RAY_AMD_SETUP_HOOK"] = str(allr["worker_process_setup_hook"])
        cwd = None
        if allr.get("working_dir"):
            cwd = allr["working_dir"]
            env["PYTHONPATH"] = cwd + os.pathsep + env["PYTHONPATH"]
        if allr.get("py_modules"):
            env["PYTHONPATH"] = os.pathsep.join(map(str, allr["py_modules"])) + os.pathsep + \
                env["PYTHONPATH"]
        cmd = [self.python, "-u", "-m", "ray_amd._private.worker_main", "--session-dir",
               self.session_dir, "--raylet", self.addr, "--token", str(w.token), "--job",
               str(job), "--node-id", node]
        if node == self.node_hex:
            w.proc = subprocess.Popen(cmd, env=env, cwd=cwd, close_fds=True,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE)
            w.pid = w.proc.pid
            self._tee_worker_logs(w)
        else:
            # the node agent forks it (its pid arrives with the worker's registration)
            self.send(self.node_recs[node]["conn"],
                      (P.REQ, 0, "spawn_worker", (w.token, cmd, env, cwd)))
        self.starting[w.token] = w
        return w

    def _dedup(self):
        d = getattr(self, "_log_dedup", None)
        if d is None:
            from ray_amd._private.log_dedup import LogDeduplicator

            d = self._log_dedup = LogDeduplicator.from_env()
        return d

    def _tee_worker_logs(self, w):
        """worker-<token>-<pid>.out/.err under <session>/logs (state API list_logs /
        get_log, CLI `logs`), each line also forwarded to this raylet's stdout / stderr
        (the driver's terminal). All pipes are drained by ONE pump thread
        (``_private/log_pump.py``), not two threads per worker."""
        import sys

        pump = getattr(self, "_log_pump", None)
        if pump is None:
            from ray_amd._private.log_pump import LogPump

            pump = self._log_pump = LogPump(self._dedup())
        d = os.path.join(self.session_dir, "logs")
        os.makedirs(d, exist_ok=True)
        to_driver = os.environ.get("RAY_AMD_LOG_TO_DRIVER", "1") != "0"
        for pipe, ext, out in ((w.proc.stdout, "out", sys.stdout), (w.proc.stderr, "err",
                                                                       sys.stderr)):
            path = os.path.join(d, f"worker-{w.token}-{w.pid}.{ext}")
            pump.add(pipe, path, out if to_driver else None, w.pid)

    def _take_idle(self, key):
        lst = self.idle.get(key)
        while lst:
            w = lst.pop()
            if w.state == "idle" and w.conn is not None:
                return w
        return None

    def _n_starting_for(self, key):
        return sum(1 for w in self.starting.values() if w.key == key)

    # ------------------------------------------------------------------ leases
    def rpc_request_lease(self, conn, rid, req):
        self.pending.append(LeaseReq(rid, conn, req))
        self.dirty = True

    def _resolve_resources(self, req):
        res = {k: float(v) for k, v in (req.get("resources") or {}).items() if v}
        st = req.get("strategy")
        if isinstance(st, dict) and st.get("type") == "pg":
            pg = st["pg_id"]
            idx = st.get("bundle_index", -1)
            out = {}
            for k, v in res.items():
                out[f"{k}_group_{pg}"] = v
                if idx is not None and idx >= 0:
                    out[f"{k}_group_{idx}_{pg}"] = v
            if idx is not None and idx >= 0:
                out[f"bundle_group_{idx}_{pg}"] = 0.001
            else:
                out[f"bundle_group_{pg}"] = 0.001
            return out
        return res

    @staticmethod
    def _lease_shape(req):
        """(strategy code, target node, hard labels, soft labels, class key) of a lease
        request: everything pick_node needs besides the resources."""
        st = req.get("strategy")
        strategy, target = 0, ""
        hard_l, soft_l = {}, {}
        if st == "SPREAD":
            strategy = 1
        elif isinstance(st, dict):
            if st.get("type") == "node_affinity":
                strategy = 3 if st.get("soft") else 2
                target = st["node_id"]
            elif st.get("type") == "node_label":
                hard_l = {k: ",".join(v) if isinstance(v, (list, tuple)) else str(v)
                          for k, v in (st.get("hard") or {}).items()}
                soft_l = {k: ",".join(v) if isinstance(v, (list, tuple)) else str(v)
                          for k, v in (st.get("soft") or {}).items()}
        res = req.get("resources") or {}
        skey = (tuple(sorted((k, float(v)) for k, v in res.items() if v)), repr(st))
        return strategy, target, hard_l, soft_l, skey

    def try_schedule(self):
        if not self.pending:
            return
        keep = collections.deque()
        starting_budget = self.max_starting - len(self.starting)
        # scheduling classes that found no room in this pass: later requests of the same
        # class wait without another pick (the owners keep up to 64 lease requests per
        # class pending, so a full node would otherwise be re-searched for each of them;
        # reference: cluster_task_manager.cc skips a scheduling class once it is blocked)
        blocked = set()
        while self.pending:
            lr = self.pending.popleft()
            if lr.conn is not None and lr.conn not in self.conn_worker and lr.cb is None:
                # requester gone
                if lr.alloc is not None:
                    self.sched.release(lr.alloc, lr.resources)
                continue
            if lr.alloc is None:
                if lr.shape is None:
                    lr.resources = self._resolve_resources(lr.req)
                    lr.shape = self._lease_shape(lr.req)
                res = lr.resources
                st = lr.req.get("strategy")
                strategy, target, hard_l, soft_l, skey = lr.shape
                rw = self.conn_worker.get(lr.conn)
                local = rw.node if rw is not None and rw.node else self.node_hex
                bkey = (skey, local)
                if bkey in blocked:
                    keep.append(lr)
                    continue
                node = self.sched.pick_node(res, strategy, target, local, hard_l, soft_l)
                if node == "!":
                    if isinstance(st, dict) and st.get("type") == "pg" and (
                            st["pg_id"] not in self.pgs or
                            self.pgs[st["pg_id"]].state == "REMOVED"):
                        self._fail_lease(lr, "placement group was removed", pg_removed=True)
                        continue
                    if not lr.warned:
                        lr.warned = True
                        print(f"[ray_amd] warning: task/actor {lr.req.get('name')} requires "
                              f"{res} which no node can satisfy; it stays pending.",
                              file=sys.stderr, flush=True)
                    keep.append(lr)
                    continue
                if node == "":
                    blocked.add(bkey)
                    keep.append(lr)
                    continue
                alloc = self.sched.allocate(node, res)
                if alloc is None:
                    blocked.add(bkey)
                    keep.append(lr)
                    continue
                lr.alloc = alloc
                lr.node = node
            if not self.node_recs.get(lr.node, {}).get("alive"):
                lr.alloc = None  # node died after allocation: pick again
                keep.append(lr)
                continue
            gpu_ids = self._gpu_ids(lr.alloc)
            key = self._pool_key(lr.req.get("job"), lr.req.get("runtime_env"), gpu_ids,
                                 lr.node, self._shared_visible(lr, gpu_ids))
            w = self._take_idle(key)
            if w is None:
                if lr.waiting_token is None or lr.waiting_token not in self.starting:
                    if starting_budget > 0 or self._n_starting_for(key) == 0:
                        nw = self._start_worker(key, lr.req.get("runtime_env"),
                                                lr.req.get("job"))
                        lr.waiting_token = nw.token
                        starting_budget -= 1
                keep.append(lr)
                continue
            self._grant(lr, w, gpu_ids)
        self.pending = keep

    def _gpu_ids(self, alloc):
        inst = alloc.instances
        if not inst:
            return []
        best = None
        for name, lst in inst.items():
            if best is None or len(name) > len(best):
                best = name
        return sorted(i for i, _ in inst[best])

    def _grant(self, lr, w, gpu_ids):
        lid = self.next_lease
        self.next_lease += 1
        lease = Lease(lid, w, lr.alloc, lr.resources, lr.req.get("owner"), lr.req.get("strategy"),
                      lr.req.get("retriable", True))
        st = lr.req.get("strategy")
        if isinstance(st, dict) and st.get("type") == "pg":
            lease.pg = st["pg_id"]
        self.leases[lid] = lease
        w.state = "leased"
        w.lease = lease
        grant = {"addr": w.addr, "lease_id": lid, "gpu_ids": gpu_ids, "worker_id": w.wid,
                 "pid": w.pid, "node_id": w.node}
        if lr.cb is not None:
            lr.cb(grant)
        else:
            self.reply(lr.conn, lr.rid, True, grant)

    def _fail_lease(self, lr, msg, pg_removed=False):
        from ray_amd.exceptions import (ActorPlacementGroupRemoved, TaskPlacementGroupRemoved,
                                        TaskUnschedulableError)

        if pg_removed:  # lr.cb is set for actor-creation leases, None for task leases
            err = (ActorPlacementGroupRemoved if lr.cb is not None else
                   TaskPlacementGroupRemoved)(msg)
        else:
            err = TaskUnschedulableError(msg)
        if lr.cb is not None:
            lr.cb(None, err)
        else:
            self.reply(lr.conn, lr.rid, False, err)

    def rpc_return_lease(self, conn, rid, lid, worker_dead):
        self._return_lease(lid, kill=worker_dead)
        self.reply(conn, rid, True, None)

    def _return_lease(self, lid, kill=False):
        lease = self.leases.pop(lid, None)
        if lease is None:
            return
        res = dict(lease.resources)
        if lease.cpu_released:
            res.pop("CPU", None)
        self.sched.release(lease.alloc, res)
        w = lease.worker
        w.lease = None
        if kill or w.actor_id is not None:
            self._kill_worker(w)
        elif w.conn is not None:
            w.state = "idle"
            w.idle_since = time.monotonic()
            self.idle[w.key].append(w)
        self.dirty = True

    def rpc_notify_blocked(self, conn, rid, wid):
        w = self.workers.get(wid)
        if w is None or w.lease is None or w.lease.cpu_released:
            return
        cpu = w.lease.resources.get("CPU")
        if cpu:
            # give the CPU back while the task waits in ray.get (avoids nested-task deadlock)
            self.sched.release(self._node_alloc(w.node), {"CPU": cpu})
            w.lease.cpu_released = True
            self.dirty = True

    def rpc_notify_unblocked(self, conn, rid, wid):
        w = self.workers.get(wid)
        if w is None or w.lease is None or not w.lease.cpu_released:
            return
        cpu = w.lease.resources.get("CPU")
        if cpu and self.sched.allocate(w.node, {"CPU": cpu}) is not None:
            w.lease.cpu_released = False

    def _node_alloc(self, node):
        a = self.sched.allocate(node, {})
        return a

    # ------------------------------------------------------------------ worker death
    def on_closed(self, conn):
        addr = self.conn_addr.pop(conn, None)
        if addr:
            self.addr_conn.pop(addr, None)
        nh = self.node_conn.pop(conn, None)
        if nh is not None:
            self._on_node_dead(nh)
            return
        w = self.conn_worker.pop(conn, None)
        if w is None:
            return
        w.conn = None
        self.workers.pop(w.wid, None)
        if w.mode == "driver":
            self._on_driver_exit(w)
            return
        prev_state = w.state
        w.state = "dead"
        if w.lease is not None:
            lease = w.lease
            self.leases.pop(lease.lid, None)
            res = dict(lease.resources)
            if lease.cpu_released:
                res.pop("CPU", None)
            self.sched.release(lease.alloc, res)
            w.lease = None
        if w.proc is not None:
            try:
                w.proc.wait(timeout=0.5)
            except Exception:
                pass
        self._release_store_pins(w)
        if w.actor_id is not None:
            cause = getattr(w, "death_cause", None)
            a = self.actors.get(w.actor_id)
            if a is not None and cause and cause.startswith("oom:"):
                a._oom_cause = ("The actor died because its node ran out of memory. "
                                + cause.split(":", 2)[2])
            self._on_actor_worker_died(w.actor_id, prev_state)
        self.dirty = True

    def _release_store_pins(self, w):
        """Zero-copy views / unsealed creates of a dead worker must not pin store memory
        forever (its process can no longer release them)."""
        if not w.pid:
            return
        try:
            if w.node == self.node_hex:
                self.store.release_all_pins_of(int(w.pid))
            else:
                rec = self.node_recs.get(w.node)
                if rec and rec["alive"] and rec.get("conn") is not None:
                    self.send(rec["conn"], (P.REQ, 0, "release_pins_of", (int(w.pid),)))
        except Exception:
            traceback.print_exc()

    def _kill_worker(self, w, graceful=False):
        w.state = "dead"
        if w.conn is not None:
            try:
                self.send(w.conn, (P.PUSH, "exit", None))
            except Exception:
                pass
        if w.proc is not None:
            try:
                if not graceful:
                    w.proc.kill()
            except Exception:
                pass
        elif w.node != self.node_hex and w.node in self.node_recs:
            rec = self.node_recs[w.node]
            if rec["alive"] and w.pid:
                self.send(rec["conn"], (P.REQ, 0, "kill_worker", (w.pid, graceful)))
        elif w.pid:
            try:
                os.kill(w.pid, signal.SIGKILL)
            except OSError:
                pass

    def _on_driver_exit(self, w):
        j = self.jobs.get(w.job)
        if j:
            j["status"] = "SUCCEEDED"
            j["end_time"] = time.time()
            self._gcs_dirty = True
        # leases held by the driver: kill those workers (they may run its tasks)
        for lid, lease in list(self.leases.items()):
            if lease.owner == w.addr:
                self._return_lease(lid, kill=True)
        for aid, a in list(self.actors.items()):
            if a.info.get("owner") == w.addr and a.info.get("lifetime") != "detached":
                self._kill_actor(a, no_restart=True, reason="owner (driver) exited")
        for pg in list(self.pgs.values()):
            if pg.owner == w.addr and pg.lifetime != "detached":
                self._remove_pg(pg)
        # idle workers of this job are useless now
        for key, lst in list(self.idle.items()):
            if key[0] == w.job:
                for iw in lst:
                    self._kill_worker(iw)
                lst.clear()

    # ------------------------------------------------------------------ periodic
    def _memory_check(self, now):
        if self.mem_monitor is None or now - self._mem_last < self.mem_refresh:
            return
        self._mem_last = now
        if self._oom_victim is not None:
            w, deadline = self._oom_victim
            if w.state != "dead" and now < deadline:
                return  # give the last victim time to exit before killing again
            self._oom_victim = None
        used, total, src = self.mem_monitor.snapshot()
        if not self.mem_monitor.over_threshold(used, total):
            return
        cands = [l for l in self.leases.values()
                 if l.worker is not None and l.worker.node == self.node_hex and
                 l.worker.mode == "worker" and l.worker.state != "dead" and l.worker.pid]
        lease, retry = select_worker_to_kill(cands, self.kill_policy)
        if lease is None:
            return
        w = lease.worker
        rss = self.mem_monitor.process_private_bytes(int(w.pid))
        msg = (f"Task was killed due to the node running low on memory. Memory on the node "
               f"({src}) was {used / 2**30:.2f}GB / {total / 2**30:.2f}GB "
               f"({used / max(total, 1):.3f}), which exceeds the memory usage threshold of "
               f"{self.mem_monitor.threshold}. ray_amd killed this worker (pid={w.pid}, "
               f"private memory {max(rss, 0) / 2**30:.2f}GB) because it was the most recent "
               f"{'retriable ' if lease.retriable else ''}lease of the policy "
               f"'{self.kill_policy}' choice. Set RAY_memory_usage_threshold / "
               f"RAY_memory_monitor_refresh_ms=0 to tune or disable.")
        print(f"[ray_amd] memory monitor: {msg}", file=sys.stderr, flush=True)
        # the policy's retry verdict travels with the cause: a lease alone in its owner
        # group is failed with OutOfMemoryError instead of being re-killed on every retry
        cause = "oom:" + ("retry:" if retry else "noretry:") + msg
        self.death_causes[w.addr] = cause
        while len(self.death_causes) > 1000:
            self.death_causes.popitem(last=False)
        w.death_cause = cause
        self.oom_kills += 1
        self._oom_victim = (w, now + 5.0)
        self._kill_worker(w)

    def rpc_death_cause(self, conn, rid, addr):
        """Why a worker died, if the raylet killed it ("oom:retry:<message>" or
        "oom:noretry:<message>")."""
        self.reply(conn, rid, True, self.death_causes.get(addr))

    # ------------------------------------------------------------------ GCS durability
    def _gcs_file(self):
        return os.path.join(self._gcs_path, "gcs_snapshot.pkl")

    def _gcs_snapshot(self):
        """A copy of the durable tables, taken on the loop thread (values the loop mutates
        later — job records — are copied; KV values are immutable bytes)."""
        actors = [{"info": a.info, "spec": a.spec, "restarts": a.restarts,
                   "node": a.worker.node if a.worker is not None else
                   getattr(a, "readopt_node", None)}
                  for a in self.actors.values()
                  if a.info.get("lifetime") == "detached" and a.state != P.DEAD]
        pgs = [{"pg_id": pg.pg_id, "bundles": pg.bundles, "strategy": pg.strategy,
                "name": pg.name, "lifetime": pg.lifetime, "namespace": pg.namespace}
               for pg in self.pgs.values()
               if pg.lifetime == "detached" and pg.state != "REMOVED"]
        return {"version": 1, "kv": dict(self.kv),
                "jobs": {k: dict(v) for k, v in self.jobs.items()},
                "job_counter": self.job_counter, "actors": actors, "pgs": pgs,
                "head": self.node_hex, "saved_at": time.time()}

    def _gcs_write(self, snap):
        import pickle

        tmp = self._gcs_file() + f".tmp{os.getpid()}"
        try:
            with open(tmp, "wb") as f:
                pickle.dump(snap, f, protocol=5)
            os.replace(tmp, self._gcs_file())
        except Exception:  # noqa: BLE001
            traceback.print_exc()

    def _gcs_save(self, sync=False):
        """Persist the snapshot. The loop thread only copies the tables; pickling and the
        file write run on a background writer (one at a time: while one is in flight the
        tables stay dirty and the next tick saves again), so a large KV — Serve checkpoints,
        runtime_env packages — does not stall the head's control loop. ``sync`` (shutdown)
        waits for an in-flight writer and writes inline."""
        w = self._gcs_writer
        if w is not None and w.is_alive():
            if not sync:
                return
            w.join()
        snap = self._gcs_snapshot()
        self._gcs_dirty = False
        self._gcs_saved = time.monotonic()
        if sync:
            self._gcs_write(snap)
            return
        self._gcs_writer = threading.Thread(target=self._gcs_write, args=(snap,),
                                            name="gcs-snapshot", daemon=True)
        self._gcs_writer.start()

    def _gcs_restore(self):
        import pickle

        path = self._gcs_file()
        if not os.path.exists(path):
            return
        with open(path, "rb") as f:  # written by _gcs_save of an earlier head (our own file)
            st = pickle.load(f)
        self.kv.update(st.get("kv") or {})
        now = time.time()
        for jid, j in (st.get("jobs") or {}).items():
            j = dict(j)
            if j.get("status") == "RUNNING":  # its driver died with the previous head
                j["status"] = "FAILED"
                j["end_time"] = j.get("end_time") or now
                j["message"] = "the head node restarted"
            self.jobs[jid] = j
        self.job_counter = max([self.job_counter, int(st.get("job_counter") or 0)] +
                               [int(k) for k in self.jobs])
        for d in st.get("pgs") or []:
            pg = PGRec(d["pg_id"], d["bundles"], d["strategy"], d["name"], d["lifetime"], None,
                       d["namespace"])
            self.pgs[pg.pg_id] = pg
            if pg.name:
                self.pg_names[(pg.namespace, pg.name)] = pg.pg_id
        for d in st.get("actors") or []:
            a = ActorRec(d["info"], d["spec"])
            a.restarts = int(d.get("restarts") or 0)
            self.actors[a.aid] = a
            node = d.get("node")
            if node and node != st.get("head") and self._readopt_grace > 0:
                # it ran on a worker node, whose agent and workers may outlive the head:
                # wait for its worker to re-attach before re-creating it
                a.state = P.RESTARTING
                a.readopt_node = node
                self._readopt[a.aid] = (a, time.monotonic() + self._readopt_grace)
                if a.info.get("name"):
                    self.named[(a.info.get("namespace"), a.info["name"])] = a.aid
                continue
            self._restart_restored(a, now)
        self.gcs_restored = {"kv": len(st.get("kv") or {}), "jobs": len(st.get("jobs") or {}),
                             "actors": len(st.get("actors") or []),
                             "pgs": len(st.get("pgs") or []),
                             "awaiting_reattach": len(self._readopt)}
        self._gcs_dirty = True

    def _restart_restored(self, a, now):
        """A restored detached actor whose process died with the previous head (or did not
        re-attach in time): re-create it if it has restarts left (the head restart killed
        the actor's process: that is a restart like any other, so an actor that has used
        its max_restarts stays dead)."""
        if a.max_restarts != -1 and a.restarts >= a.max_restarts:
            a.state = P.DEAD
            a.death = ("The actor died with the head node and has no restarts left "
                       f"(max_restarts={a.max_restarts}).")
            a.end_time = now
            return
        a.restarts += 1
        a.state = P.RESTARTING
        if a.info.get("name"):
            self.named[(a.info.get("namespace"), a.info["name"])] = a.aid
        self._schedule_actor(a)
        self._gcs_dirty = True

    def rpc_reattach_actor(self, conn, rid, aid):
        """A surviving worker re-attaches its actor to this (restarted) head (reference:
        raylet NodeManager::HandleNotifyGCSRestart → workers re-subscribe; the GCS actor
        table keeps the actor ALIVE at its address). The worker registered on this
        connection first; its node agent must have re-registered too. Replies True
        (adopted), "retry" (its node is not back yet) or False (exit: the actor was
        re-created, removed or was never durable)."""
        w = self.conn_worker.get(conn)
        ent = self._readopt.get(aid)
        a = ent[0] if ent else None
        if w is None or a is None or a.worker is not None or a.state == P.DEAD:
            self.reply(conn, rid, True, False)
            return
        rec = self.node_recs.get(w.node)
        if rec is None or not rec["alive"] or w.node == self.node_hex:
            self.reply(conn, rid, True, "retry")
            return
        res = {k: float(v) for k, v in (a.spec.get("resources") or {}).items()}
        alloc = self.sched.allocate(w.node, res)
        if alloc is None:
            self.reply(conn, rid, True, False)
            return
        lid = self.next_lease
        self.next_lease += 1
        lease = Lease(lid, w, alloc, res, self.addr, a.spec.get("strategy"),
                      a.max_restarts != 0)
        lease.actor_id = aid
        self.leases[lid] = lease
        w.state = "actor"
        w.lease = lease
        w.actor_id = aid
        w.job = a.spec.get("job")
        a.worker, a.lease, a.pid = w, lease, w.pid
        a.state = P.ALIVE
        self._readopt.pop(aid, None)
        self._publish(a)
        self._gcs_dirty = True
        self.dirty = True
        print(f"[ray_amd] actor {a.info.get('class_name')} re-attached from node "
              f"{w.node[:12]} (pid {w.pid})", file=sys.stderr, flush=True)
        self.reply(conn, rid, True, True)

    def _readopt_expired(self, now_m):
        for aid, (a, deadline) in list(self._readopt.items()):
            if a.worker is not None or a.state == P.DEAD:
                self._readopt.pop(aid, None)
            elif now_m > deadline:
                self._readopt.pop(aid, None)
                self._restart_restored(a, time.time())

    def rpc_gcs_status(self, conn, rid):
        self.reply(conn, rid, True, {"storage_path": self._gcs_path,
                                     "restored": self.gcs_restored})

    def tick(self):
        now = time.monotonic()
        if self._readopt:
            self._readopt_expired(now)
        if self._gcs_path and self._gcs_dirty and now - self._gcs_saved > 0.2:
            self._gcs_save()
        self._memory_check(now)
        for pg in self.pgs.values():
            if pg.state == "PENDING":
                self._try_place(pg)
        # reap idle workers beyond the soft limit
        n_idle = sum(len(v) for v in self.idle.values())
        if n_idle > self.num_cpus:
            for key, lst in self.idle.items():
                for w in list(lst):
                    if n_idle <= self.num_cpus:
                        break
                    if now - w.idle_since > 2.0:
                        lst.remove(w)
                        self._kill_worker(w, graceful=True)
                        n_idle -= 1
        # workers that failed to start
        for tok, w in list(self.starting.items()):
            if w.proc is not None and w.proc.poll() is not None:
                self.starting.pop(tok, None)
                print(f"[ray_amd] worker process {w.pid} exited during startup "
                      f"(code {w.proc.returncode})", file=sys.stderr, flush=True)
                self.dirty = True

    # ------------------------------------------------------------------ kv
    def rpc_kv_put(self, conn, rid, ns, key, value, overwrite=True):
        self._gcs_dirty = True
        k = (ns, key)
        existed = k in self.kv
        if overwrite or not existed:
            self.kv[k] = value
        self.reply(conn, rid, True, not existed)

    def rpc_kv_get(self, conn, rid, ns, key):
        self.reply(conn, rid, True, self.kv.get((ns, key)))

    def rpc_kv_del(self, conn, rid, ns, key, prefix=False):
        self._gcs_dirty = True
        if prefix:
            ks = [k for k in self.kv if k[0] == ns and _startswith(k[1], key)]
            for k in ks:
                del self.kv[k]
            self.reply(conn, rid, True, len(ks))
        else:
            self.reply(conn, rid, True, 1 if self.kv.pop((ns, key), None) is not None else 0)

    def rpc_kv_keys(self, conn, rid, ns, prefix):
        self.reply(conn, rid, True, [k[1] for k in self.kv if k[0] == ns and
                                     _startswith(k[1], prefix)])

    def rpc_kv_exists(self, conn, rid, ns, key):
        self.reply(conn, rid, True, (ns, key) in self.kv)

    # ------------------------------------------------------------------ actors
    def rpc_create_actor(self, conn, rid, info, spec):
        name = info.get("name")
        ns = info.get("namespace")
        if name:
            existing = self.named.get((ns, name))
            if existing is not None and self.actors[existing].state != P.DEAD:
                if info.get("get_if_exists"):
                    a = self.actors[existing]
                    self.reply(conn, rid, True, {"existing": existing,
                                                 "method_meta": a.spec.get("method_meta"),
                                                 "class_name": a.info.get("class_name"),
                                                 "owner": a.info.get("owner")})
                    return
                self.reply(conn, rid, False, ValueError(
                    f"The name {name} (namespace={ns}) is already taken. Please use a "
                    f"different name or get the existing actor using ray.get_actor('{name}')"))
                return
        a = ActorRec(info, spec)
        self.actors[a.aid] = a
        if name:
            self.named[(ns, name)] = a.aid
        self._schedule_actor(a)
        self._gcs_dirty = True
        self.reply(conn, rid, True, None)

    def _schedule_actor(self, a):
        req = {"resources": a.spec.get("resources") or {}, "strategy": a.spec.get("strategy"),
               "runtime_env": a.spec.get("runtime_env"), "owner": self.addr,
               "job": a.spec.get("job"), "name": a.info.get("class_name"),
               "retriable": a.max_restarts != 0}

        def granted(grant, err=None, a=a):
            if grant is None:
                self._actor_dead(a, str(err))
                return
            if a.state == P.DEAD:
                self._return_lease(grant["lease_id"], kill=False)
                return
            lease = self.leases[grant["lease_id"]]
            lease.actor_id = a.aid
            w = lease.worker
            w.actor_id = a.aid
            w.state = "actor"
            a.worker = w
            a.lease = lease
            a.pid = w.pid
            spec = dict(a.spec)
            spec["lease_id"] = grant["lease_id"]
            self.send(w.conn, (P.TASK, spec))

        self.pending.append(LeaseReq(0, None, req, cb=granted))
        self.dirty = True

    def on_task_reply(self, conn, msg):
        _, tid, returns, extra = msg
        w = self.conn_worker.get(conn)
        if w is None or w.actor_id is None:
            return
        a = self.actors.get(w.actor_id)
        if a is None:
            return
        if returns and returns[0][0] == "__init_error__":
            a.no_restart = True
            self._actor_dead(a, ("err", returns[0][1]))
            self._kill_worker(w)
            return
        a.state = P.ALIVE
        if a.info.get("lifetime") == "detached":
            self._gcs_dirty = True  # its node goes into the snapshot (re-attach on restart)
        self._publish(a)

    def _publish(self, a):
        death = a.death
        if isinstance(death, tuple) and death and death[0] == "err":
            try:
                _, exc = ser.deserialize(death[1])
                death = exc
            except Exception:
                death = "actor creation failed"
        msg = (P.PUSH, "actor", (a.aid, a.state, a.worker.addr if a.worker and
                                 a.state == P.ALIVE else None, death, a.restarts))
        for c in list(a.subscribers):
            if c in self.conn_worker:
                self.send(c, msg)
            else:
                a.subscribers.discard(c)

    def rpc_subscribe_actor(self, conn, rid, aid):
        a = self.actors.get(aid)
        if a is None:
            self.reply(conn, rid, True, (aid, P.DEAD, None, "actor not found", 0))
            return
        a.subscribers.add(conn)
        death = a.death
        if isinstance(death, tuple):
            try:
                _, death = ser.deserialize(death[1])
            except Exception:
                death = "actor creation failed"
        self.reply(conn, rid, True, (aid, a.state, a.worker.addr if a.worker and
                                     a.state == P.ALIVE else None, death, a.restarts))

    def _on_actor_worker_died(self, aid, prev_state):
        a = self.actors.get(aid)
        if a is None or a.state == P.DEAD:
            return
        a.worker = None
        a.lease = None
        can_restart = not a.no_restart and (a.max_restarts == -1 or a.restarts < a.max_restarts)
        if can_restart:
            a.restarts += 1
            a.state = P.RESTARTING
            self._publish(a)
            self._schedule_actor(a)
        else:
            cause = getattr(a, "_oom_cause", None)
            self._actor_dead(a, cause if cause else
                             "The actor died unexpectedly (worker process exited)."
                             if not a.no_restart else "The actor was killed (ray.kill).")

    def _actor_dead(self, a, death):
        self._gcs_dirty = True
        a.state = P.DEAD
        a.death = death
        a.end_time = time.time()
        self._publish(a)

    def _kill_actor(self, a, no_restart=True, reason="ray.kill"):
        a.no_restart = a.no_restart or no_restart
        if a.worker is not None:
            w = a.worker
            if a.lease is not None:
                self.leases.pop(a.lease.lid, None)
                res = dict(a.lease.resources)
                self.sched.release(a.lease.alloc, res)
                w.lease = None
                a.lease = None
            self._kill_worker(w)
            if no_restart:
                self._actor_dead(a, f"The actor was killed ({reason}).")
                a.worker = None
        elif no_restart:
            self._actor_dead(a, f"The actor was killed ({reason}).")
        self.dirty = True

    def rpc_kill_actor(self, conn, rid, aid, no_restart):
        a = self.actors.get(aid)
        if a is not None:
            self._kill_actor(a, no_restart)
        self.reply(conn, rid, True, a is not None)

    def rpc_actor_out_of_scope(self, conn, rid, aid):
        a = self.actors.get(aid)
        if a is not None and a.info.get("lifetime") != "detached" and not a.info.get("name"):
            self._kill_actor(a, True, "all handles out of scope")

    def rpc_actor_exit(self, conn, rid, aid):
        a = self.actors.get(aid)
        if a is not None:
            a.no_restart = True
            self._actor_dead(a, "The actor exited via exit_actor().")

    def rpc_get_named_actor(self, conn, rid, name, namespace):
        aid = self.named.get((namespace, name))
        if aid is None or self.actors[aid].state == P.DEAD:
            self.reply(conn, rid, True, None)
            return
        a = self.actors[aid]
        self.reply(conn, rid, True, {"actor_id": aid, "method_meta": a.spec.get("method_meta"),
                                     "class_name": a.info.get("class_name"),
                                     "owner": a.info.get("owner")})

    def rpc_list_named_actors(self, conn, rid, all_namespaces, namespace):
        out = []
        for (ns, name), aid in self.named.items():
            if self.actors[aid].state == P.DEAD:
                continue
            if all_namespaces:
                out.append({"name": name, "namespace": ns})
            elif ns == namespace:
                out.append(name)
        self.reply(conn, rid, True, out)

    def rpc_list_actors(self, conn, rid):
        out = []
        for aid, a in self.actors.items():
            out.append({"actor_id": aid.hex(), "class_name": a.info.get("class_name"),
                        "state": a.state, "name": a.info.get("name") or "",
                        "namespace": a.info.get("namespace"), "pid": a.pid,
                        "num_restarts": a.restarts, "job_id": a.spec.get("job"),
                        "node_id": self.node_id.hex(),
                        "death_cause": a.death if isinstance(a.death, str) else
                        ("creation task error" if a.death else None),
                        "lifetime": a.info.get("lifetime") or "non_detached",
                        "required_resources": a.spec.get("resources"),
                        "start_time": a.start_time, "end_time": a.end_time})
        self.reply(conn, rid, True, out)

    # ------------------------------------------------------------------ placement groups
    def rpc_create_pg(self, conn, rid, pg_id, bundles, strategy, name, lifetime, owner,
                      namespace):
        if name and (namespace, name) in self.pg_names:
            self.reply(conn, rid, False, ValueError(f"placement group name {name} exists"))
            return
        pg = PGRec(pg_id, bundles, strategy, name, lifetime, owner, namespace)
        self.pgs[pg_id] = pg
        self._gcs_dirty = True
        if name:
            self.pg_names[(namespace, name)] = pg_id
        self._try_place(pg)
        self.reply(conn, rid, True, None)

    def _try_place(self, pg):
        if pg.state != "PENDING":
            return
        nodes, infeasible = self.sched.place_bundles(
            [{k: float(v) for k, v in b.items()} for b in pg.bundles],
            _PG_STRATEGY.get(pg.strategy, 0))
        if not nodes:
            if infeasible:
                pg.state = "PENDING"  # stays pending (reference behaviour), flagged infeasible
                pg.infeasible = True
            return
        if self.sched.commit_bundles(pg.pg_id, [{k: float(v) for k, v in b.items()}
                                                for b in pg.bundles], nodes):
            pg.nodes = nodes
            pg.state = "CREATED"
            for conn, rid in pg.waiters:
                self.reply(conn, rid, True, True)
            pg.waiters.clear()
            self.dirty = True

    def rpc_wait_pg(self, conn, rid, pg_id):
        pg = self.pgs.get(pg_id)
        if pg is None:
            self.reply(conn, rid, False, ValueError("placement group does not exist"))
            return
        if pg.state == "CREATED":
            self.reply(conn, rid, True, True)
        elif pg.state == "REMOVED":
            self.reply(conn, rid, False, ValueError("placement group was removed"))
        else:
            pg.waiters.append((conn, rid))

    def rpc_remove_pg(self, conn, rid, pg_id):
        pg = self.pgs.get(pg_id)
        if pg is not None:
            self._remove_pg(pg)
        self.reply(conn, rid, True, None)

    def _remove_pg(self, pg):
        if pg.state == "REMOVED":
            return
        self._gcs_dirty = True
        # kill workers leased inside the pg
        for lid, lease in list(self.leases.items()):
            if lease.pg == pg.pg_id:
                if lease.actor_id is not None and lease.actor_id in self.actors:
                    self._kill_actor(self.actors[lease.actor_id], True, "placement group removed")
                else:
                    self._return_lease(lid, kill=True)
        if pg.state == "CREATED":
            self.sched.remove_bundles(pg.pg_id, [{k: float(v) for k, v in b.items()}
                                                 for b in pg.bundles], pg.nodes)
        pg.state = "REMOVED"
        pg.removed_at = time.time()
        for conn, rid in pg.waiters:
            self.reply(conn, rid, False, ValueError("placement group was removed"))
        pg.waiters.clear()
        if pg.name:
            self.pg_names.pop((pg.namespace, pg.name), None)
        self.dirty = True

    def rpc_pg_table(self, conn, rid, pg_id):
        def rec(pg):
            return {"placement_group_id": pg.pg_id, "name": pg.name or "",
                    "bundles": {i: b for i, b in enumerate(pg.bundles)},
                    "bundles_to_node_id": {i: n for i, n in enumerate(pg.nodes)},
                    "strategy": pg.strategy, "state": pg.state,
                    "stats": {"scheduling_state": "FINISHED" if pg.state == "CREATED"
                              else "PENDING"}}
        if pg_id is not None:
            pg = self.pgs.get(pg_id)
            self.reply(conn, rid, True, rec(pg) if pg else None)
        else:
            self.reply(conn, rid, True, {k: rec(v) for k, v in self.pgs.items()})

    def rpc_get_named_pg(self, conn, rid, name, namespace):
        pid = self.pg_names.get((namespace, name))
        if pid is None:
            self.reply(conn, rid, True, None)
            return
        pg = self.pgs[pid]
        self.reply(conn, rid, True, {"pg_id": pid, "bundles": pg.bundles,
                                     "strategy": pg.strategy})

    # ------------------------------------------------------------------ cluster info
    def rpc_cluster_resources(self, conn, rid):
        tot = self.sched.cluster_total()
        self.reply(conn, rid, True, {k: v for k, v in tot.items() if "_group_" not in k})

    def rpc_available_resources(self, conn, rid):
        av = self.sched.cluster_available()
        self.reply(conn, rid, True, {k: v for k, v in av.items()
                                     if "_group_" not in k and v > 0})

    def rpc_nodes(self, conn, rid):
        out = []
        for nh, rec in self.node_recs.items():
            res = self.sched.total(nh) if rec["alive"] else dict(rec["resources"])
            out.append({
                "NodeID": nh, "Alive": rec["alive"], "NodeManagerAddress": self.node_ip,
                "NodeManagerHostname": os.uname().nodename,
                "Resources": {k: v for k, v in res.items() if "_group_" not in k},
                "alive": rec["alive"], "RayletSocketName": rec["addr"],
                "ObjectStoreSocketName": rec["store_path"], "Labels": rec["labels"],
                "node_id": nh, "is_head_node": rec.get("is_head", False)})
        self.reply(conn, rid, True, out)

    def rpc_resource_load(self, conn, rid):
        """Autoscaler input (reference: GcsResourceManager load report / autoscaler
        LoadMetrics): resource shapes waiting for a node, pending placement-group
        bundles, and per-node usage with an idle-since timestamp."""
        demand = []
        for lr in self.pending:
            if lr.alloc is None:
                r = {k: float(v) for k, v in (lr.req.get("resources") or {}).items() if v}
                st = lr.req.get("strategy")
                if not (isinstance(st, dict) and st.get("type") == "pg"):
                    demand.append(r)
        pg_demand = [[{k: float(v) for k, v in b.items()} for b in pg.bundles]
                     for pg in self.pgs.values() if pg.state == "PENDING"]
        now = time.time()
        busy = collections.Counter(l.worker.node for l in self.leases.values()
                                   if l.worker is not None)
        nodes = []
        for nh, rec in self.node_recs.items():
            if not rec["alive"]:
                continue
            tot = {k: v for k, v in self.sched.total(nh).items() if "_group_" not in k}
            av = {k: v for k, v in self.sched.available(nh).items() if "_group_" not in k}
            idle = busy.get(nh, 0) == 0 and all(av.get(k, 0) >= v - 1e-9 for k, v in tot.items())
            if idle:
                rec.setdefault("idle_since", now)
            else:
                rec.pop("idle_since", None)
            nodes.append({"node_id": nh, "total": tot, "available": av,
                          "is_head": rec.get("is_head", False), "labels": rec["labels"],
                          "idle_s": now - rec["idle_since"] if idle else 0.0,
                          "num_leases": busy.get(nh, 0)})
        req = self.kv.get(("__autoscaler", b"resource_request"))
        self.reply(conn, rid, True, {"demand": demand, "pg_demand": pg_demand, "nodes": nodes,
                                     "requested": req})

    def rpc_fetch_object(self, conn, rid, oid):
        """Serve a copy of an object held in this node's store (object_manager Pull)."""
        self.reply(conn, rid, True, read_object_bytes(self.store, self.spill_dir, oid))

    def rpc_fetch_object_chunk(self, conn, rid, oid, off, n):
        """One chunk of an object (object_manager chunked Pull)."""
        self.reply(conn, rid, True, read_object_chunk(self.store, self.spill_dir, oid, off, n))

    def rpc_free_objects(self, conn, rid, oids):
        for oid in oids:
            free_object(self.store, self.spill_dir, oid)
        self.reply(conn, rid, True, None)

    def rpc_node_addr(self, conn, rid, node_hex):
        rec = self.node_recs.get(node_hex)
        self.reply(conn, rid, True, rec["addr"] if rec is not None and rec["alive"] else None)

    # ------------------------------------------------------------------ cluster membership
    def rpc_register_node(self, conn, rid, node_hex, total, labels, addr, store_path,
                          spill_dir, pid, ncpu):
        """A worker-node agent joins (reference: GcsNodeManager::HandleRegisterNode)."""
        labels = dict(labels)
        labels.setdefault("ray.io/node_id", node_hex)
        self.sched.add_node(node_hex, total, labels)
        self.node_recs[node_hex] = {
            "node_id": node_hex, "addr": addr, "conn": conn, "store_path": store_path,
            "spill_dir": spill_dir, "labels": labels, "resources": dict(total),
            "alive": True, "pid": pid, "is_head": False, "start_time": time.time(),
            "num_cpus": ncpu}
        self.node_conn[conn] = node_hex
        self.num_cpus += ncpu
        self.max_starting = max(self.max_starting, 4, self.num_cpus)
        for pg in list(self.pgs.values()):
            self._try_place(pg)
        self.dirty = True
        self.reply(conn, rid, True, {"head_node_id": self.node_hex})

    def _on_node_dead(self, nh):
        """Node agent connection lost: remove the node (reference: OnNodeFailure)."""
        rec = self.node_recs.get(nh)
        if rec is None or not rec["alive"]:
            return
        rec["alive"] = False
        rec["end_time"] = time.time()
        self.num_cpus -= rec.get("num_cpus", 0)
        print(f"[ray_amd] node {nh[:12]} died", file=sys.stderr, flush=True)
        for tok, w in list(self.starting.items()):
            if w.node == nh:
                self.starting.pop(tok, None)
        for w in list(self.workers.values()):
            if w.node == nh and w.conn is not None:
                # its socket will close too; do not wait for that to free the actor/lease
                self.on_closed(w.conn)
        for lst in self.idle.values():
            lst[:] = [w for w in lst if w.node != nh]
        for pg in self.pgs.values():
            if pg.state == "CREATED" and nh in pg.nodes:
                # bundles on the dead node are gone: reschedule the whole group
                self.sched.remove_bundles(pg.pg_id, [{k: float(v) for k, v in b.items()}
                                                     for b in pg.bundles], pg.nodes)
                pg.state = "PENDING"
                pg.nodes = []
        self.sched.remove_node(nh)
        for pg in list(self.pgs.values()):
            self._try_place(pg)
        self.dirty = True

    def rpc_list_workers(self, conn, rid):
        out = []
        for w in self.workers.values():
            out.append({"worker_id": w.wid.hex(), "pid": w.pid, "worker_type": w.mode,
                        "state": w.state, "job_id": w.job, "actor_id": w.actor_id.hex()
                        if w.actor_id else None, "gpu_ids": list(w.gpu_ids)})
        self.reply(conn, rid, True, out)

    def rpc_list_jobs(self, conn, rid):
        self.reply(conn, rid, True, list(self.jobs.values()))

    _TASK_RANK = {"PENDING_ARGS_AVAIL": 0, "PENDING_NODE_ASSIGNMENT": 1, "SUBMITTED_TO_WORKER": 2,
                  "RUNNING": 3, "FINISHED": 4, "FAILED": 4}
    _TASK_TYPES = {P.NORMAL_TASK: "NORMAL_TASK", P.ACTOR_TASK: "ACTOR_TASK",
                   P.ACTOR_CREATION_TASK: "ACTOR_CREATION_TASK"}

    def rpc_task_events(self, conn, rid, events):
        """Task lifecycle events from owners (submission) and executors (running / done).
        Merged per (task, attempt) into the state table behind `ray_amd.util.state`
        (reference: core_worker/task_event_buffer.cc → gcs_task_manager.cc)."""
        table = self.task_table
        rank = self._TASK_RANK
        for ev in events:
            tid, name, t0, t1, pid, aid, status = ev[:7]
            ttype, job, attempt, err = ev[7:11] if len(ev) >= 11 else (None, None, 0, None)
            if t1 is not None:
                self.task_events.append(ev)
            key = (tid, attempt)
            rec = table.get(key)
            if rec is None:
                rec = table[key] = {
                    "task_id": tid.hex(), "attempt_number": attempt, "name": name,
                    "func_or_class_name": name, "state": status,
                    "job_id": job.hex() if isinstance(job, bytes) else job,
                    "actor_id": aid.hex() if aid else None,
                    "type": self._TASK_TYPES.get(ttype, "NORMAL_TASK"),
                    "node_id": self.node_id.hex(), "worker_pid": None, "error_type": None,
                    "creation_time_ms": int(t0 * 1000), "start_time_ms": None,
                    "end_time_ms": None, "language": "PYTHON"}
                if len(table) > 200000:
                    table.popitem(last=False)
            if rank.get(status, 0) >= rank.get(rec["state"], 0):
                rec["state"] = status
            if pid is not None:
                rec["worker_pid"] = pid
            if status == "RUNNING" or (t1 is not None and rec["start_time_ms"] is None):
                rec["start_time_ms"] = int(t0 * 1000)
            if t1 is not None:
                rec["end_time_ms"] = int(t1 * 1000)
                rec["error_type"] = err
            if aid and not rec["actor_id"]:
                rec["actor_id"] = aid.hex()

    def rpc_metrics(self, conn, rid, pid, snapshot):
        self.app_metrics[pid] = snapshot

    def rpc_get_metrics(self, conn, rid):
        """Application metric snapshots of every process + node/system series
        (reference: metrics agent + ray_* system metrics in metric_defs.cc)."""
        node = (("NodeId", self.node_id.hex()),)
        states = collections.Counter(r["state"] for r in self.task_table.values())
        actors = collections.Counter(a.state for a in self.actors.values())
        workers = collections.Counter(w.state for w in self.workers.values())
        tot = self.sched.cluster_total()
        av = self.sched.cluster_available()
        sysm = [
            {"kind": "gauge", "name": "ray_tasks", "description": "Tasks by state",
             "series": {node + (("State", k),): float(v) for k, v in states.items()}},
            {"kind": "gauge", "name": "ray_actors", "description": "Actors by state",
             "series": {node + (("State", k),): float(v) for k, v in actors.items()}},
            {"kind": "gauge", "name": "ray_workers", "description": "Worker processes by state",
             "series": {node + (("State", k),): float(v) for k, v in workers.items()}},
            {"kind": "gauge", "name": "ray_object_store_memory",
             "description": "Object store bytes in use",
             "series": {node: float(self.store.used(-1))}},
            {"kind": "gauge", "name": "ray_object_store_capacity",
             "description": "Object store capacity bytes",
             "series": {node: float(self.store.capacity(-1))}},
            {"kind": "gauge", "name": "ray_object_store_num_objects",
             "description": "Objects in the store", "series": {node: float(self.store.num_objects())}},
            {"kind": "gauge", "name": "ray_resources_total", "description": "Node resources",
             "series": {node + (("Name", k),): float(v) for k, v in tot.items()
                        if "_group_" not in k}},
            {"kind": "gauge", "name": "ray_resources_available",
             "description": "Available node resources",
             "series": {node + (("Name", k),): float(v) for k, v in av.items()
                        if "_group_" not in k}},
        ]
        out = list(sysm)
        from ray_amd._private.reporter import metric_records

        out.extend(metric_records(self._node_samples()))
        for snap in self.app_metrics.values():
            out.extend(snap)
        self.reply(conn, rid, True, out)

    def _node_samples(self):
        own = self.reporter.latest() or self.reporter.sample()
        alive = {nh for nh, rec in self.node_recs.items() if rec["alive"]}
        return [own] + [s for nh, s in self.node_stats.items() if nh in alive]

    def rpc_report_node_stats(self, conn, rid, node_hex, sample):
        """A node agent's periodic telemetry sample."""
        self.node_stats[node_hex] = sample
        self.reply(conn, rid, True, None)

    def rpc_node_stats(self, conn, rid):
        """node hex -> latest telemetry sample (state API / dashboard / ray_amd status)."""
        out = {}
        for s in self._node_samples():
            if s:
                out[s["node_id"]] = s
        self.reply(conn, rid, True, out)

    def rpc_list_tasks(self, conn, rid):
        self.reply(conn, rid, True, list(self.task_table.values()))

    def rpc_get_task_events(self, conn, rid):
        self.reply(conn, rid, True, list(self.task_events))

    def rpc_store_stats(self, conn, rid):
        self.reply(conn, rid, True, {"used": self.store.used(-1),
                                     "capacity": self.store.capacity(-1),
                                     "num_objects": self.store.num_objects()})

    def rpc_list_objects(self, conn, rid):
        out = []
        for o in self.store.list():
            out.append({"object_id": o["id"].hex(), "object_size": o["data_size"],
                        "pinned": o["pinned"], "ref_count": o["ref_count"],
                        "device": o["device"], "node_id": self.node_id.hex()})
        self.reply(conn, rid, True, out)

    def rpc_ping(self, conn, rid):
        self.reply(conn, rid, True, "pong")

    # ------------------------------------------------------------------ GPU arenas
    def rpc_gpu_arena(self, conn, rid, device, size):
        """HBM object store arena for `device` (allocated by a holder process so the raylet
        itself never initialises HIP)."""
        a = self.gpu_arenas.get(device)
        if a is None:
            a = self._start_arena_holder(device, size)
        self.reply(conn, rid, True, a)

    def _start_arena_holder(self, device, size):
        import tempfile

        out = os.path.join(self.session_dir, f"arena_{device}.json")
        env = dict(os.environ)
        pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = pkg_root + os.pathsep + env.get("PYTHONPATH", "")
        sock = os.path.join(self.session_dir, "sockets", f"arena_{device}.sock")
        proc = subprocess.Popen([self.python, "-m", "ray_amd._private.gpu_object_store",
                                 "--device", str(device), "--size", str(size), "--out", out,
                                 "--store", self.store_path, "--sock", sock], env=env,
                                close_fds=True)
        t0 = time.time()
        while not os.path.exists(out):
            if proc.poll() is not None or time.time() - t0 > 120:
                raise RuntimeError(f"GPU arena holder for device {device} failed")
            time.sleep(0.05)
        with open(out) as f:
            info = json.load(f)
        info["pid"] = proc.pid
        self.gpu_arenas[device] = info
        self._arena_procs = getattr(self, "_arena_procs", []) + [proc]
        tempfile  # noqa: B018
        return info

    # ------------------------------------------------------------------ shutdown
    def rpc_shutdown(self, conn, rid):
        self.reply(conn, rid, True, None)
        self.stop = True

    def shutdown(self):
        if self._gcs_path:
            self._gcs_save(sync=True)
        for w in list(self.workers.values()) + list(self.starting.values()):
            if w.mode != "driver":
                self._kill_worker(w)
        for lst in self.idle.values():
            for w in lst:
                self._kill_worker(w)
        for p in getattr(self, "_arena_procs", []):
            try:
                p.kill()
            except Exception:
                pass
        self.spiller.stop()
        shm_segment.release(self.store_path, self._store_fd)
        self.io.stop()


def read_object_bytes(store, spill_dir, oid):
    """Bytes of a sealed object in a node's shm store (or its spill file), else None."""
    b = store.get_buffer(oid, True)
    if b is not None:
        mv = memoryview(b)
        try:
            return bytes(mv)
        finally:
            mv.release()
            b.release()
    p, off, size = _spill_range(store, spill_dir, oid)
    try:
        with open(p, "rb") as f:
            f.seek(off)
            return f.read(size) if size is not None else f.read()
    except OSError:
        return None


def _spill_range(store, spill_dir, oid):
    """(file, offset, size) of a spilled object: its fused-file range (stub), else the
    per-object fallback file (size None = whole file)."""
    from .object_store import spilled_location

    loc = spilled_location(store, spill_dir, oid)
    if loc is not None:
        return loc
    return os.path.join(spill_dir, oid.hex()), 0, None


def read_object_chunk(store, spill_dir, oid, off, n):
    """(total size, bytes [off, off + n)) of a sealed object, or None (chunked pulls)."""
    b = store.get_buffer(oid, True)
    if b is not None:
        mv = memoryview(b)
        try:
            total = len(mv)
            return total, bytes(mv[off:min(total, off + n)])
        finally:
            mv.release()
            b.release()
    p, base, size = _spill_range(store, spill_dir, oid)
    try:
        with open(p, "rb") as f:
            total = os.fstat(f.fileno()).st_size if size is None else size
            f.seek(base + off)
            return total, f.read(max(0, min(n, total - off)))
    except OSError:
        return None


def free_object(store, spill_dir, oid):
    from .object_store import stub_id

    store.remove(oid)
    store.remove(stub_id(oid))  # a spilled object's stub (its fused file is GC'd)
    try:
        os.unlink(os.path.join(spill_dir, oid.hex()))
    except OSError:
        pass


def _startswith(k, prefix):
    if isinstance(k, bytes) and isinstance(prefix, str):
        prefix = prefix.encode()
    if isinstance(k, str) and isinstance(prefix, bytes):
        prefix = prefix.decode()
    return k.startswith(prefix)


def _picklable(e):
    try:
        P.dumps(e)
        return True
    except Exception:
        return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--session-dir", required=True)
    ap.add_argument("--store-path", required=True)
    ap.add_argument("--object-store-memory", type=int, default=2 << 30)
    ap.add_argument("--num-cpus", type=int, default=None)
    ap.add_argument("--num-gpus", type=int, default=None)
    ap.add_argument("--memory", type=int, default=None)
    ap.add_argument("--resources", default="{}")
    ap.add_argument("--labels", default="{}")
    ap.add_argument("--head", action="store_true")
    ap.add_argument("--head-address", default=None,
                    help="join an existing cluster as a worker node (head raylet socket)")
    ap.add_argument("--ready-file", default="raylet.ready")
    ap.add_argument("--fate-share-pid", type=int, default=0,
                    help="exit (graceful shutdown) once this process is gone")
    args = ap.parse_args()
    if args.head_address:
        from .node_agent import NodeAgent

        r = NodeAgent(args)
    else:
        r = Raylet(args)
    signal.signal(signal.SIGTERM, lambda *_: setattr(r, "stop", True))
    if args.fate_share_pid:
        import threading

        def _watch(pid=args.fate_share_pid):
            while not r.stop:
                time.sleep(1.0)
                try:
                    os.kill(pid, 0)
                except ProcessLookupError:
                    r.stop = True  # the run loop shuts the node down (workers, store file)
                    return
                except PermissionError:
                    pass

        threading.Thread(target=_watch, name="fate-share", daemon=True).start()
    ready = os.path.join(args.session_dir, args.ready_file)
    with open(ready + ".tmp", "w") as f:
        json.dump({"addr": r.addr, "node_id": r.node_id.hex(), "pid": os.getpid()}, f)
    os.replace(ready + ".tmp", ready)
    r.run()


if __name__ == "__main__":
    main()
