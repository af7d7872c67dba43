"""GCS restart with live re-adopt (reference: src/ray/raylet/node_manager.cc:1096-1110
HandleNotifyGCSRestart, src/ray/core_worker/core_worker.cc re-subscription; the GCS FT
tests kill and restart the GCS while raylets and actors keep running).

With RAY_AMD_GCS_STORAGE_PATH, a head crash no longer takes the worker nodes down: their
agents keep their object stores and workers and re-register with the restarted head on
the same socket, and a detached actor living on such a node re-attaches ITSELF — same
process, same in-memory state, no restart counted. An actor that does not come back
within the grace period is re-created from its spec as before."""
import os
import time

import pytest

import ray_amd as ray
from ray_amd.cluster_utils import Cluster


@ray.remote
class Counter:
    def __init__(self, start=0):
        self.n = start

    def inc(self):
        self.n += 1
        return self.n

    def pid(self):
        return os.getpid()


@pytest.fixture
def ft_cluster(tmp_path, monkeypatch):
    monkeypatch.setenv("RAY_AMD_GCS_STORAGE_PATH", str(tmp_path / "gcs"))
    monkeypatch.setenv("RAY_AMD_GCS_READOPT_S", "20")
    c = Cluster(initialize_head=True, head_node_args={"num_cpus": 1})
    yield c
    if ray.is_initialized():
        ray.shutdown()
    c.shutdown()


def test_worker_node_actor_survives_head_restart(ft_cluster):
    cluster = ft_cluster
    node = cluster.add_node(num_cpus=2, resources={"pool": 2})
    cluster.connect(namespace="ft")
    c = Counter.options(name="ctr", namespace="ft", lifetime="detached",
                        resources={"pool": 1}).remote(10)
    assert ray.get(c.inc.remote()) == 11
    pid = ray.get(c.pid.remote())
    time.sleep(0.8)  # the snapshot (with the actor's node) is written within 0.2 s

    cluster.restart_head()
    assert node.alive()  # the worker-node agent rode out the head crash
    cluster.connect(namespace="ft")
    from ray_amd.util.state import list_actors

    c2 = ray.get_actor("ctr", namespace="ft")
    assert ray.get(c2.inc.remote(), timeout=60) == 12  # same process, state kept
    assert ray.get(c2.pid.remote()) == pid
    acts = [a for a in list_actors() if a["name"] == "ctr"]
    assert acts and acts[0]["state"] == "ALIVE" and acts[0]["num_restarts"] == 0
    # the re-registered node schedules new work, and its resources account for the actor
    ok = Counter.options(resources={"pool": 1}).remote()
    assert ray.get(ok.inc.remote(), timeout=60) == 1
    ray.kill(c2)


def test_actor_not_reattached_is_recreated(ft_cluster, monkeypatch):
    """The worker node died with the head: after the grace period the actor is
    re-created from its creation spec on a node that has its resources."""
    monkeypatch.setenv("RAY_AMD_GCS_READOPT_S", "1")
    cluster = ft_cluster
    node = cluster.add_node(num_cpus=1, resources={"pool": 1})
    cluster.connect(namespace="ft")
    c = Counter.options(name="ctr2", namespace="ft", lifetime="detached", max_restarts=1,
                        resources={"pool": 1}).remote(5)
    assert ray.get(c.inc.remote()) == 6
    time.sleep(0.8)
    cluster.remove_node(node, allow_graceful=False)
    cluster.restart_head()
    cluster.add_node(num_cpus=1, resources={"pool": 1})
    cluster.connect(namespace="ft")
    c2 = ray.get_actor("ctr2", namespace="ft")
    assert ray.get(c2.inc.remote(), timeout=60) == 6  # re-created: state from the spec
    ray.kill(c2)
