"""Serve ProxyLocation.EveryNode (modelled on python/ray/serve/tests/test_proxy_state.py and
test_cluster.py): one HTTP proxy per alive node of a cluster_utils.Cluster, started as
nodes join and stopped as they leave; every proxy routes to the application."""

import socket
import time

import requests

import ray_amd as ray
from ray_amd import serve
from ray_amd.cluster_utils import Cluster
from ray_amd.serve.api import HTTPOptions
from ray_amd.serve.config import ProxyLocation
from ray_amd.serve.schema import ServeDeploySchema


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _proxies(timeout=30, want=None):
    c = serve.api._get_controller()
    deadline = time.time() + timeout
    out = {}
    while time.time() < deadline:
        out = ray.get(c.get_proxies.remote())
        if (want is None or len(out) == want) and all(v["ready"] for v in out.values()):
            return out
        time.sleep(0.3)
    return out


def test_every_node_proxies_follow_node_membership():
    port = _free_port()
    c = Cluster(initialize_head=True, head_node_args={"num_cpus": 2})
    n1 = c.add_node(num_cpus=1)
    ray.init(address=c.address)
    try:
        serve.start(http_options=HTTPOptions(port=port, location="EveryNode"))

        @serve.deployment
        class Echo:
            def __call__(self, req):
                return "hi"

        serve.run(Echo.bind(), route_prefix="/echo")
        px = _proxies(want=2)
        assert len(px) == 2, px
        ports = sorted(v["port"] for v in px.values())
        assert len(set(ports)) == 2  # one machine: the second proxy got its own port
        for p in ports:  # every node's proxy serves the app
            for _ in range(50):
                try:
                    r = requests.get(f"http://127.0.0.1:{p}/echo", timeout=5)
                    if r.status_code == 200:
                        break
                except requests.ConnectionError:
                    pass
                time.sleep(0.2)
            assert r.status_code == 200 and r.text.strip('"') == "hi"
        n2 = c.add_node(num_cpus=1)  # a node joins: it gets a proxy
        px = _proxies(want=3)
        assert len(px) == 3
        c.remove_node(n2)  # and loses it when it leaves
        px = _proxies(want=2)
        assert len(px) == 2 and n2.node_id not in px
        assert n1.node_id in px
    finally:
        serve.shutdown()
        ray.shutdown()
        c.shutdown()


def test_proxy_location_maps_through_schema():
    cfg = ServeDeploySchema(applications=[], proxy_location="EveryNode")
    assert ProxyLocation(cfg.proxy_location) == ProxyLocation.EveryNode
    assert HTTPOptions(location="EveryNode").location == "EveryNode"
