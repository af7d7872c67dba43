"""Serve tests (modelled on python/ray/serve/tests/test_api.py, test_batching.py,
test_autoscaling_policy.py, test_handle*.py, test_fastapi.py)."""

import asyncio
import time

import pytest
import requests

import ray_amd as ray
from ray_amd import serve


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=8)
    serve.start(http_options={"port": 18123})
    yield
    serve.shutdown()
    ray.shutdown()


def test_function_and_class_deployments(cluster):
    @serve.deployment
    def hello(request):
        return {"msg": "hello " + request.query_params.get("name", "x")}

    serve.run(hello.bind(), name="fn", route_prefix="/hello")
    r = requests.get("http://127.0.0.1:18123/hello?name=amd", timeout=10)
    assert r.status_code == 200 and r.json() == {"msg": "hello amd"}

    @serve.deployment(num_replicas=2)
    class Model:
        def __init__(self, k):
            self.k = k

        def __call__(self, x):
            return x * self.k

        def other(self, x):
            return x + self.k

    h = serve.run(Model.bind(3), name="m", route_prefix=None)
    assert h.remote(5).result() == 15
    assert h.other.remote(5).result() == 8
    assert serve.status()["m"]["deployments"]["Model"]["replica_states"]["RUNNING"] == 2


def test_composition(cluster):
    @serve.deployment
    class Pre:
        def __call__(self, x):
            return x + 1

    @serve.deployment
    class Ingress:
        def __init__(self, pre):
            self.pre = pre

        async def __call__(self, x):
            y = await self.pre.remote(x)
            return y * 10

    h = serve.run(Ingress.bind(Pre.bind()), name="comp", route_prefix=None)
    assert h.remote(1).result() == 20


def test_batching(cluster):
    @serve.deployment
    class Batched:
        def __init__(self):
            self.sizes = []

        @serve.batch(max_batch_size=8, batch_wait_timeout_s=0.1)
        async def __call__(self, xs):
            self.sizes.append(len(xs))
            return [x * 2 for x in xs]

        def get_sizes(self):
            return self.sizes

    h = serve.run(Batched.bind(), name="b", route_prefix=None)
    resps = [h.remote(i) for i in range(16)]
    assert [r.result() for r in resps] == [i * 2 for i in range(16)]
    assert max(h.get_sizes.remote().result()) > 1


def test_user_config_reconfigure(cluster):
    @serve.deployment(user_config={"t": 1})
    class C:
        def reconfigure(self, cfg):
            self.t = cfg["t"]

        def __call__(self):
            return self.t

    h = serve.run(C.bind(), name="cfg", route_prefix=None)
    assert h.remote().result() == 1
    h = serve.run(C.options(user_config={"t": 7}).bind(), name="cfg", route_prefix=None)
    time.sleep(0.3)
    assert h.remote().result() == 7


def test_autoscaling(cluster):
    @serve.deployment(autoscaling_config={"min_replicas": 1, "max_replicas": 3,
                                          "target_ongoing_requests": 1,
                                          "upscale_delay_s": 0.2, "downscale_delay_s": 0.5},
                      max_ongoing_requests=10)
    class Slow:
        async def __call__(self):
            await asyncio.sleep(1.0)
            return 1

    h = serve.run(Slow.bind(), name="auto", route_prefix=None)
    resps = [h.remote() for _ in range(12)]
    deadline = time.time() + 10
    n = 1
    while time.time() < deadline:
        n = serve.status()["auto"]["deployments"]["Slow"]["replica_states"]["RUNNING"]
        if n > 1:
            break
        time.sleep(0.2)
    [r.result() for r in resps]
    assert n > 1


def test_fastapi_ingress(cluster):
    from fastapi import FastAPI

    app = FastAPI()

    @serve.deployment
    @serve.ingress(app)
    class Api:
        def __init__(self):
            self.n = 41

        @app.get("/answer")
        def answer(self):
            return {"answer": self.n + 1}

    serve.run(Api.bind(), name="api", route_prefix="/api")
    r = requests.get("http://127.0.0.1:18123/api/answer", timeout=10)
    assert r.status_code == 200 and r.json() == {"answer": 42}, r.text
    serve.delete("api")
    assert "api" not in serve.status()
