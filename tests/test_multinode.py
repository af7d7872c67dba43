"""Multi-node cluster tests on one machine (modelled on python/ray/tests/
test_multi_node*.py, test_scheduling*.py, test_placement_group_*.py and
test_object_manager.py, which drive ray.cluster_utils.Cluster)."""

import time

import numpy as np
import pytest

import ray_amd as ray
from ray_amd.cluster_utils import Cluster
from ray_amd.exceptions import RayActorError
from ray_amd.util.placement_group import placement_group, placement_group_table
from ray_amd.util.scheduling_strategies import (NodeAffinitySchedulingStrategy,
                                                NodeLabelSchedulingStrategy)


@pytest.fixture
def cluster3():
    c = Cluster(initialize_head=True, head_node_args={"num_cpus": 1})
    n1 = c.add_node(num_cpus=2, resources={"a": 1}, labels={"zone": "z1"})
    n2 = c.add_node(num_cpus=2, resources={"b": 1}, labels={"zone": "z2"})
    ray.init(address=c.address)
    yield c, n1, n2
    ray.shutdown()
    c.shutdown()


@ray.remote
def where():
    return ray.get_runtime_context().get_node_id()


@ray.remote
def total(x):
    return float(np.asarray(x).sum()), ray.get_runtime_context().get_node_id()


@ray.remote
def make(n):
    return np.ones(n)


def test_nodes_join_and_resources(cluster3):
    c, n1, n2 = cluster3
    nodes = ray.nodes()
    assert len(nodes) == 3 and all(n["Alive"] for n in nodes)
    assert {n["NodeID"] for n in nodes} == {c.head_node.node_id, n1.node_id, n2.node_id}
    res = ray.cluster_resources()
    assert res["CPU"] == 5 and res["a"] == 1 and res["b"] == 1


def test_custom_resource_affinity_and_labels(cluster3):
    c, n1, n2 = cluster3
    assert ray.get(where.options(resources={"a": 1}).remote()) == n1.node_id
    assert ray.get(where.options(resources={"b": 1}).remote()) == n2.node_id
    st = NodeAffinitySchedulingStrategy(n2.node_id, soft=False)
    assert ray.get(where.options(scheduling_strategy=st).remote()) == n2.node_id
    st = NodeLabelSchedulingStrategy(hard={"zone": "z1"})
    assert ray.get(where.options(scheduling_strategy=st).remote()) == n1.node_id


def test_spread_uses_several_nodes(cluster3):
    @ray.remote
    def slow_where():
        time.sleep(0.3)
        return ray.get_runtime_context().get_node_id()

    ids = ray.get([slow_where.options(scheduling_strategy="SPREAD").remote()
                   for _ in range(5)])
    assert len(set(ids)) == 3


def test_cross_node_objects(cluster3):
    c, n1, n2 = cluster3
    big = ray.put(np.arange(1_000_000, dtype=np.float64))  # head-node store
    s, node = ray.get(total.options(resources={"b": 1}).remote(big))
    assert node == n2.node_id and s == float(np.arange(1_000_000).sum())
    r = make.options(resources={"a": 1}).remote(500_000)  # primary copy on node a
    assert ray.get(r).sum() == 500_000  # driver pulls it to the head node
    s, node = ray.get(total.options(resources={"b": 1}).remote(r))  # b pulls it from a
    assert node == n2.node_id and s == 500_000


def test_remote_actor_and_node_death(cluster3):
    c, n1, n2 = cluster3

    @ray.remote(max_restarts=0)
    class A:
        def node(self):
            return ray.get_runtime_context().get_node_id()

        def arr(self):
            return np.zeros(300_000)

    a = A.options(resources={"b": 1}).remote()
    assert ray.get(a.node.remote()) == n2.node_id
    assert ray.get(a.arr.remote()).shape == (300_000,)
    c.remove_node(n2)
    alive = {n["NodeID"] for n in ray.nodes() if n["Alive"]}
    assert n2.node_id not in alive
    with pytest.raises(RayActorError):
        ray.get(a.node.remote(), timeout=20)
    # the cluster keeps scheduling on the survivors
    assert ray.get(where.options(resources={"a": 1}).remote()) == n1.node_id


def test_strict_spread_pg_and_late_node(cluster3):
    c, n1, n2 = cluster3
    pg = placement_group([{"CPU": 1}] * 3, strategy="STRICT_SPREAD")
    assert ray.get(pg.ready(), timeout=20)
    placed = placement_group_table(pg)["bundles_to_node_id"]
    assert len(set(placed.values())) == 3
    from ray_amd.util.placement_group import remove_placement_group

    remove_placement_group(pg)
    # 4 strict-spread bundles need a 4th node: pending until it joins
    pg4 = placement_group([{"CPU": 1}] * 4, strategy="STRICT_SPREAD")
    time.sleep(0.5)
    assert placement_group_table(pg4)["state"] == "PENDING"
    c.add_node(num_cpus=1)
    assert ray.get(pg4.ready(), timeout=20)


def test_large_object_pulled_in_chunks(cluster3):
    """A 48 MB object made on another node arrives intact through chunked parallel pulls
    (reference: object_manager chunked transfers, test_object_manager.py)."""
    c, n1, n2 = cluster3
    from ray_amd._private import worker as W

    cw = W.global_worker.core
    old = cw.PULL_CHUNK
    cw.PULL_CHUNK = 4 << 20  # force 12 chunks
    try:
        ref = make.options(resources={"b": 1}).remote(6 << 20)  # 6M float64 = 48 MB
        arr = ray.get(ref)
        assert arr.shape == (6 << 20,) and float(arr.sum()) == float(6 << 20)
    finally:
        cw.PULL_CHUNK = old


def test_label_selector(cluster3):
    """label_selector (reference: ray.remote(label_selector=...)): equality, negation,
    in() / !in() lists; a node without the label matches a negated selector."""
    c, n1, n2 = cluster3
    head = c.head_node.node_id
    assert ray.get(where.options(label_selector={"zone": "z2"}).remote()) == n2.node_id
    assert ray.get(where.options(label_selector={"zone": "in(z1,z9)"}).remote()) == n1.node_id
    got = {ray.get(where.options(label_selector={"zone": "!z1"}).remote()) for _ in range(8)}
    assert n1.node_id not in got and got <= {n2.node_id, head}
    got = {ray.get(where.options(label_selector={"zone": "!in(z1,z2)"}).remote())
           for _ in range(4)}
    assert got == {head}
    with pytest.raises(ValueError):
        where.options(label_selector={"zone": "in()"}).remote()
    with pytest.raises(ValueError):
        where.options(label_selector={"zone": "z1"}, scheduling_strategy="SPREAD").remote()


def test_worker_logs_on_other_nodes(cluster3):
    """A worker forked by a node agent gets worker-<token>-<pid>.out under the session's
    logs directory, drained by the agent's LogPump (reference: log_monitor.py runs per
    node)."""
    import glob
    import os
    import time

    c, n1, n2 = cluster3

    @ray.remote(resources={"b": 1})
    def shout():
        print("hello-from-node-b", flush=True)
        return ray.get_runtime_context().get_node_id()

    assert ray.get(shout.remote()) != ray.get(where.options(resources={"a": 1}).remote())
    deadline = time.time() + 10
    hit = []
    while time.time() < deadline and not hit:
        for f in glob.glob(os.path.join(c.session_dir, "logs", "worker-*.out")):
            with open(f, "rb") as fh:
                if b"hello-from-node-b" in fh.read():
                    hit.append(f)
        time.sleep(0.1)
    assert hit
