"""Multi-node clusters on one machine (reference: python/ray/cluster_utils.py:135 Cluster).

The first ``add_node`` starts the head raylet (scheduler + GCS tables + the head
node's object store); every later ``add_node`` starts a worker-node agent
(``_private/node_agent.py``) that registers with the head, hosts its own shm object
store and spawns that node's workers. Objects move between nodes by pull
(``fetch_object``) into the reader's store, exactly as between real hosts; only the
transport (Unix-domain sockets) is single-machine.

    cluster = Cluster(initialize_head=True, head_node_args={"num_cpus": 2})
    cluster.add_node(num_cpus=2, resources={"pool": 1})
    ray.init(address=cluster.address)
"""

from __future__ import annotations

import atexit
import json
import os
import subprocess
import sys
import time

import ray_amd
from ray_amd._private import worker as _W

_DEFAULT_OSM = 256 << 20


class Node:
    """Handle on one started node process (head raylet or worker-node agent)."""

    def __init__(self, proc, node_id, address, is_head, args):
        self.proc = proc
        self.node_id = node_id
        self.unique_id = node_id
        self.address = address
        self.is_head = is_head
        self.node_args = args

    def alive(self) -> bool:
        return self.proc.poll() is None

    def kill(self, graceful=True):
        if self.proc.poll() is not None:
            return
        if graceful:
            self.proc.terminate()
            try:
                self.proc.wait(timeout=10)
                return
            except subprocess.TimeoutExpired:
                pass
        self.proc.kill()
        self.proc.wait(timeout=10)

    def __repr__(self):
        return f"Node({'head' if self.is_head else 'worker'}, {self.node_id[:12]})"


class Cluster:
    def __init__(self, initialize_head: bool = False, connect: bool = False,
                 head_node_args: dict | None = None, shutdown_at_exit: bool = True):
        self.head_node: Node | None = None
        self.worker_nodes: set = set()
        self.session_dir: str | None = None
        self.connected = False
        self._n = 0
        if not initialize_head and connect:
            raise RuntimeError("Cannot connect to uninitialized cluster.")
        if shutdown_at_exit:
            atexit.register(self.shutdown)
        if initialize_head:
            self.add_node(**(head_node_args or {}))
            if connect:
                self.connect()

    @property
    def address(self):
        return self.session_dir

    gcs_address = address

    def connect(self, namespace=None):
        assert self.address is not None and not self.connected
        info = ray_amd.init(address=self.address, namespace=namespace,
                            ignore_reinit_error=True)
        self.connected = True
        return info

    def add_node(self, wait: bool = True, num_cpus=1, num_gpus=0, resources=None,
                 labels=None, object_store_memory=_DEFAULT_OSM, **kwargs) -> Node:
        args = dict(num_cpus=num_cpus, num_gpus=num_gpus, resources=resources or {},
                    labels=labels or {}, object_store_memory=object_store_memory)
        if self.head_node is None:
            self.session_dir = _W.new_session_dir()
            self._head_start = (num_cpus, num_gpus, resources, int(object_store_memory),
                                labels)
            proc, addr = _W._start_raylet(self.session_dir, *self._head_start)
            with open(os.path.join(self.session_dir, "raylet.ready")) as f:
                nid = json.load(f)["node_id"]
            self.head_node = Node(proc, nid, addr, True, args)
            return self.head_node
        self._n += 1
        ready = f"node_{self._n}.ready"
        store = f"/dev/shm/ray_amd_{os.path.basename(self.session_dir)}_n{self._n}"
        cmd = [sys.executable, "-m", "ray_amd._private.raylet", "--session-dir",
               self.session_dir, "--store-path", store, "--object-store-memory",
               str(int(object_store_memory)), "--resources", json.dumps(resources or {}),
               "--labels", json.dumps(labels or {}), "--num-cpus", str(int(num_cpus)),
               "--num-gpus", str(int(num_gpus or 0)), "--head-address", self.head_node.address,
               "--ready-file", ready]
        env = dict(os.environ)
        pkg_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"]
                                        if env.get("PYTHONPATH") else "")
        proc = subprocess.Popen(cmd, env=env, close_fds=True, start_new_session=True)
        path = os.path.join(self.session_dir, ready)
        t0 = time.time()
        while not os.path.exists(path):
            if proc.poll() is not None:
                raise RuntimeError(f"node agent exited with code {proc.returncode}")
            if time.time() - t0 > 60:
                proc.kill()
                raise TimeoutError("node agent did not start")
            time.sleep(0.01)
        with open(path) as f:
            info = json.load(f)
        node = Node(proc, info["node_id"], info["addr"], False, args)
        self.worker_nodes.add(node)
        if wait:
            self._wait_for_node(node)
        return node

    def _alive_ids(self):
        if not ray_amd.is_initialized():
            return None
        return {n["NodeID"] for n in ray_amd.nodes() if n["Alive"]}

    def _wait_for_node(self, node, timeout: float = 30):
        t0 = time.time()
        while time.time() - t0 < timeout:
            ids = self._alive_ids()
            if ids is None or node.node_id in ids:
                if ids is None:
                    time.sleep(0.2)  # no driver yet: give the registration a moment
                return
            time.sleep(0.05)
        raise TimeoutError(f"node {node} did not join within {timeout}s")

    def wait_for_nodes(self, timeout: float = 30):
        t0 = time.time()
        want = {n.node_id for n in self.list_all_nodes()}
        while time.time() - t0 < timeout:
            ids = self._alive_ids()
            if ids is None or want <= ids and len(ids) == len(want):
                return
            time.sleep(0.05)
        raise TimeoutError("timed out waiting for nodes to join / leave")

    def remove_node(self, node: Node, allow_graceful: bool = True):
        if node is self.head_node:
            if ray_amd.is_initialized() and self.connected:
                ray_amd.shutdown()
                self.connected = False
            node.kill(allow_graceful)
            self.head_node = None
            return
        node.kill(allow_graceful)
        self.worker_nodes.discard(node)
        t0 = time.time()
        while time.time() - t0 < 30:
            ids = self._alive_ids()
            if ids is None or node.node_id not in ids:
                return
            time.sleep(0.05)

    def restart_head(self, timeout: float = 60):
        """Kill the head raylet (SIGKILL: a crash, no goodbye to the node agents) and start
        a new one on the same session and socket. With RAY_AMD_GCS_STORAGE_PATH the new
        head reloads the persisted tables, the worker-node agents re-register and their
        detached actors re-attach with their state (reference: GCS fault tolerance tests'
        kill_gcs_server / restart_gcs_server). The driver is disconnected first; connect
        again with ``ray_amd.init(address=cluster.address)``."""
        if self.connected and ray_amd.is_initialized():
            ray_amd.shutdown()
        self.connected = False
        old = self.head_node
        old.kill(graceful=False)
        try:
            os.unlink(os.path.join(self.session_dir, "raylet.ready"))
        except FileNotFoundError:
            pass
        proc, addr = _W._start_raylet(self.session_dir, *self._head_start)
        with open(os.path.join(self.session_dir, "raylet.ready")) as f:
            nid = json.load(f)["node_id"]
        self.head_node = Node(proc, nid, addr, True, old.node_args)
        return self.head_node

    def list_all_nodes(self):
        nodes = list(self.worker_nodes)
        if self.head_node is not None:
            nodes.insert(0, self.head_node)
        return nodes

    def remaining_processes_alive(self) -> bool:
        return all(n.alive() for n in self.list_all_nodes())

    def shutdown(self):
        if self.connected and ray_amd.is_initialized():
            ray_amd.shutdown()
        self.connected = False
        # graceful first (SIGTERM: the agent kills its workers and releases its store),
        # all nodes at once, then SIGKILL whatever did not exit. Even a SIGKILLed agent
        # leaves no store behind: it is a memfd (_private/shm_segment.py)
        nodes = [n for n in self.worker_nodes if n.alive()]
        for n in nodes:
            n.proc.terminate()
        deadline = time.time() + 10
        for n in nodes:
            try:
                n.proc.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                n.kill(False)
        self.worker_nodes.clear()
        if self.head_node is not None:
            self.head_node.kill(True)
            self.head_node = None


class AutoscalingCluster:
    """A local cluster whose worker nodes are launched and removed by the autoscaler
    (reference: python/ray/cluster_utils.py AutoscalingCluster over the
    fake_multi_node provider).

        cluster = AutoscalingCluster(head_resources={"CPU": 0},
                                     worker_node_types={"cpu2": {"resources": {"CPU": 2},
                                                                 "max_workers": 2}},
                                     idle_timeout_minutes=0.05)
        cluster.start()
        ray.init(address=cluster.address)
    """

    def __init__(self, head_resources: dict, worker_node_types: dict,
                 idle_timeout_minutes: float = 1.0, max_workers: int = 20,
                 upscaling_speed: float = 1.0, update_interval_s: float = 0.5, **_):
        from ray_amd.autoscaler.autoscaler import AutoscalerConfig, NodeTypeConfig

        self.head_resources = dict(head_resources)
        types = {}
        for name, spec in worker_node_types.items():
            types[name] = NodeTypeConfig(resources=dict(spec["resources"]),
                                         min_workers=spec.get("min_workers", 0),
                                         max_workers=spec.get("max_workers", 10),
                                         node_config=dict(spec.get("node_config", {})))
        self.config = AutoscalerConfig(node_types=types, max_workers=max_workers,
                                       idle_timeout_s=idle_timeout_minutes * 60.0,
                                       upscaling_speed=upscaling_speed,
                                       update_interval_s=update_interval_s)
        self.cluster = None
        self.monitor = None
        self.autoscaler = None

    @property
    def address(self):
        return self.cluster.address if self.cluster else None

    def start(self, **_):
        from ray_amd.autoscaler.autoscaler import Monitor, StandardAutoscaler
        from ray_amd.autoscaler.node_provider import FakeMultiNodeProvider

        res = dict(self.head_resources)
        self.cluster = Cluster(initialize_head=True, head_node_args={
            "num_cpus": int(res.pop("CPU", 0)), "num_gpus": int(res.pop("GPU", 0)),
            "resources": res})
        provider = FakeMultiNodeProvider(self.cluster)

        def load():
            if not ray_amd.is_initialized():
                return {"demand": [], "pg_demand": [], "nodes": [], "requested": None}
            return _W.global_worker.core.call_raylet("resource_load", timeout=30)

        self.autoscaler = StandardAutoscaler(self.config, provider, load_fn=load)
        self.monitor = Monitor(self.autoscaler).start()
        return self

    def shutdown(self):
        if self.monitor is not None:
            self.monitor.stop()
        if self.cluster is not None:
            self.cluster.shutdown()
