"""Autoscaler with the local fake multi-node provider (modelled on
python/ray/tests/test_autoscaler_fake_multinode.py and test_resource_demand_scheduler.py)."""

import time

import pytest

import ray_amd as ray
from ray_amd.autoscaler import AutoscalerConfig, NodeTypeConfig, StandardAutoscaler
from ray_amd.autoscaler.autoscaler import pack
from ray_amd.autoscaler.sdk import request_resources
from ray_amd.cluster_utils import AutoscalingCluster


class _FakeProvider:
    def __init__(self):
        self.nodes = {}
        self.n = 0

    def non_terminated_nodes(self, f):
        return [k for k, v in self.nodes.items() if all(v.get(a) == b for a, b in f.items())]

    def create_node(self, cfg, tags, count):
        out = []
        for _ in range(count):
            self.n += 1
            self.nodes[f"n{self.n}"] = dict(tags)
            out.append(f"n{self.n}")
        return out

    def terminate_node(self, nid):
        self.nodes.pop(nid)

    def node_tags(self, nid):
        return self.nodes[nid]

    def ray_node_id(self, nid):
        return None  # never joins: counted as launching capacity


def test_packing_and_type_choice():
    bins = [{"CPU": 2}, {"CPU": 1, "GPU": 1}]
    left = pack([{"CPU": 1}, {"GPU": 1}, {"CPU": 2}, {"GPU": 1}], bins)
    assert left == [{"GPU": 1}]  # first-fit-decreasing: GPUs first, CPUs fill the rest
    cfg = AutoscalerConfig(node_types={
        "small": NodeTypeConfig({"CPU": 2}, max_workers=3),
        "gpu": NodeTypeConfig({"CPU": 8, "GPU": 8}, max_workers=1),
        "big": NodeTypeConfig({"CPU": 16}, max_workers=2)}, max_workers=4)
    prov = _FakeProvider()
    load = {"demand": [{"CPU": 1}] * 5 + [{"GPU": 1}] * 2, "pg_demand": [], "requested": None,
            "nodes": [{"node_id": "head", "total": {"CPU": 0}, "available": {}, "idle_s": 0}]}
    a = StandardAutoscaler(cfg, prov, load_fn=lambda: load)
    r = a.update()
    types = sorted(prov.nodes[n]["ray-user-node-type"] for n in r["launched"])
    # 2 GPU asks -> one gpu node (its 8 CPUs also absorb CPU asks); no CPU node needed
    assert types == ["gpu"], types
    # already-launching capacity is counted: a second round launches nothing new
    assert a.update()["launched"] == []
    # infeasible shapes are skipped, max_workers respected
    load["demand"] = [{"TPU": 1}] + [{"CPU": 16}] * 5
    r = a.update()
    assert len(prov.nodes) <= 4


@pytest.fixture
def autoscaling_cluster():
    c = AutoscalingCluster(head_resources={"CPU": 0},
                           worker_node_types={"cpu2": {"resources": {"CPU": 2},
                                                       "max_workers": 2}},
                           idle_timeout_minutes=3 / 60.0, update_interval_s=0.3)
    c.start()
    ray.init(address=c.address)
    yield c
    ray.shutdown()
    c.shutdown()


def test_scale_up_on_demand_then_down_when_idle(autoscaling_cluster):
    c = autoscaling_cluster

    @ray.remote(num_cpus=1)
    def work(i):
        time.sleep(0.5)
        return ray.get_runtime_context().get_node_id()

    # the head has no CPUs: these tasks can only run on autoscaled nodes
    nodes = set(ray.get([work.remote(i) for i in range(6)], timeout=90))
    assert 1 <= len(nodes) <= 2
    launched = [e for e in c.autoscaler.events if e[1] == "launch"]
    assert 1 <= len(launched) <= 2 and all(e[2] == "cpu2" for e in launched)
    # idle for idle_timeout (3 s): worker nodes are terminated
    deadline = time.time() + 60
    while time.time() < deadline:
        if len([n for n in ray.nodes() if n["Alive"]]) == 1:
            break
        time.sleep(0.5)
    assert len([n for n in ray.nodes() if n["Alive"]]) == 1
    assert any(e[1] == "terminate" for e in c.autoscaler.events)


def test_request_resources_scales_without_tasks(autoscaling_cluster):
    c = autoscaling_cluster
    request_resources(num_cpus=4)
    deadline = time.time() + 60
    while time.time() < deadline and ray.cluster_resources().get("CPU", 0) < 4:
        time.sleep(0.3)
    assert ray.cluster_resources().get("CPU", 0) >= 4
    request_resources()  # clear; nodes become idle and go away
    deadline = time.time() + 60
    while time.time() < deadline and ray.cluster_resources().get("CPU", 0) > 0:
        time.sleep(0.5)
    assert ray.cluster_resources().get("CPU", 0) == 0
    assert c.monitor.errors == 0
