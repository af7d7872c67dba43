"""Ray Client (modelled on python/ray/tests/test_client.py, test_client_references.py):
a client server drives a running cluster; a separate client process connects with
init("ray://host:port") and uses tasks, actors, put/get/wait, refs in arguments and
return values, named actors, kill, and reference release."""

import os
import socket
import subprocess
import sys
import textwrap
import time

import pytest

import ray_amd as ray

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def client_server():
    ctx = ray.init(num_cpus=4)
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=REPO)
    srv = subprocess.Popen([sys.executable, "-m", "ray_amd.util.client.server", "--address",
                            ctx["address"], "--port", str(port)], env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    line = srv.stdout.readline()
    assert "listening" in line, line
    yield port
    srv.kill()
    srv.wait()
    ray.shutdown()


CLIENT = textwrap.dedent("""
    import sys, numpy as np
    import ray_amd as ray
    from ray_amd.exceptions import RayTaskError, RayActorError

    ray.init("ray://127.0.0.1:%d")

    @ray.remote
    def add(a, b):
        return a + b

    @ray.remote
    def nested(x):
        return {"ref": ray.put(x * 2)}

    @ray.remote
    def boom():
        raise ValueError("client-boom")

    @ray.remote
    class Counter:
        def __init__(self, start):
            self.n = start
        def inc(self, k=1):
            self.n += k
            return self.n

    assert ray.get(add.remote(1, 2)) == 3
    x = ray.put(np.arange(10))
    assert int(ray.get(add.remote(x, 1)).sum()) == 55          # ref passed as an argument
    inner = ray.get(nested.remote(21))["ref"]                   # ref inside a return value
    assert ray.get(inner) == 42
    refs = [add.remote(i, i) for i in range(8)]
    ready, rest = ray.wait(refs, num_returns=8, timeout=30)
    assert sorted(ray.get(ready)) == [2 * i for i in range(8)] and not rest
    try:
        ray.get(boom.remote())
        raise SystemExit("expected failure")
    except ValueError as e:
        assert "client-boom" in str(e)
    c = Counter.options(name="ctr").remote(10)
    assert ray.get([c.inc.remote() for _ in range(3)]) == [11, 12, 13]
    c2 = ray.get_actor("ctr")
    assert ray.get(c2.inc.remote(5)) == 18
    assert ray.cluster_resources()["CPU"] == 4

    @ray.remote
    def gen(n):
        for i in range(n):
            yield i * i

    g = gen.options(num_returns="streaming").remote(5)
    assert [ray.get(r) for r in g] == [0, 1, 4, 9, 16]         # streaming over the client

    @ray.remote
    class Streamer:
        def items(self, n):
            for i in range(n):
                yield {"i": i}

    st = Streamer.remote()
    assert [ray.get(r)["i"] for r in st.items.options(num_returns="streaming").remote(3)] == \
        [0, 1, 2]
    ray.kill(c)
    try:
        ray.get(c.inc.remote(), timeout=20)
        raise SystemExit("expected actor death")
    except RayActorError:
        pass
    ray.shutdown()
    print("CLIENT_OK")
""")


def test_client_end_to_end(client_server):
    env = dict(os.environ, PYTHONPATH=REPO)
    env.pop("RAY_ADDRESS", None)
    r = subprocess.run([sys.executable, "-c", CLIENT % client_server], env=env,
                       capture_output=True, text=True, timeout=180)
    assert "CLIENT_OK" in r.stdout, r.stdout + r.stderr
    # the client's session released its server-side refs/actors on disconnect
    time.sleep(0.5)


CONNECT = textwrap.dedent("""
    from ray_amd.util.client_connect import connect, disconnect
    import ray_amd as ray

    info = connect("127.0.0.1:%d")
    assert "ray_version" in info

    @ray.remote
    def sq(x):
        return x * x

    assert ray.get(sq.remote(7)) == 49
    disconnect()
    assert not ray.is_initialized()
    print("CONNECT_OK")
""")


def test_client_connect_module(client_server):
    """util.client_connect.connect / disconnect (reference: python/ray/util/
    client_connect.py) over the same client server."""
    env = dict(os.environ, PYTHONPATH=REPO)
    env.pop("RAY_ADDRESS", None)
    r = subprocess.run([sys.executable, "-c", CONNECT % client_server], env=env,
                       capture_output=True, text=True, timeout=120)
    assert "CONNECT_OK" in r.stdout, r.stdout + r.stderr
