"""More Serve semantics (modelled on python/ray/serve/tests/test_api.py,
test_deploy.py, test_handle_*.py, test_multiplex.py, test_http_routes.py,
test_deployment_state / test_standalone): errors, redeploys, routing, options, deletion."""

import pytest
import requests

import ray_amd as ray
from ray_amd import serve

PORT = 18131


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=8)
    serve.start(http_options={"port": PORT})
    yield
    serve.shutdown()
    ray.shutdown()


def test_user_exception_reaches_caller_and_http_500(cluster):
    @serve.deployment
    class Bad:
        def __call__(self, x=None):
            raise ValueError("broken model")

    h = serve.run(Bad.bind(), name="bad", route_prefix="/bad")
    with pytest.raises(Exception) as ei:
        h.remote(1).result()
    assert "broken model" in str(ei.value)
    r = requests.get(f"http://127.0.0.1:{PORT}/bad", timeout=10)
    assert r.status_code == 500
    # the replica survives a user exception
    with pytest.raises(Exception):
        h.remote(2).result()
    serve.delete("bad")


def test_redeploy_updates_code_and_config(cluster):
    @serve.deployment(version="1")
    class V:
        def __call__(self):
            return "v1"

    h = serve.run(V.bind(), name="ver", route_prefix=None)
    assert h.remote().result() == "v1"

    @serve.deployment(version="2")
    class V:  # noqa: F811 (redeployed class)
        def __call__(self):
            return "v2"

    h = serve.run(V.bind(), name="ver", route_prefix=None)
    assert h.remote().result() == "v2"
    serve.delete("ver")


def test_scaling_num_replicas_by_redeploy(cluster):
    @serve.deployment(num_replicas=1)
    class R:
        def __call__(self):
            import os

            return os.getpid()

    h = serve.run(R.bind(), name="scale", route_prefix=None)
    assert len({h.remote().result() for _ in range(10)}) == 1
    h = serve.run(R.options(num_replicas=3).bind(), name="scale", route_prefix=None)
    st = serve.status()["scale"]["deployments"]["R"]["replica_states"]
    assert st.get("RUNNING") == 3
    pids = {h.remote().result() for _ in range(60)}
    assert len(pids) == 3  # requests are spread over all replicas
    serve.delete("scale")


def test_multiple_apps_and_route_prefixes(cluster):
    @serve.deployment
    def a(req):
        return "A"

    @serve.deployment
    def b(req):
        return "B"

    serve.run(a.bind(), name="app_a", route_prefix="/a")
    serve.run(b.bind(), name="app_b", route_prefix="/b")
    assert requests.get(f"http://127.0.0.1:{PORT}/a", timeout=10).text.strip('"') == "A"
    assert requests.get(f"http://127.0.0.1:{PORT}/b", timeout=10).text.strip('"') == "B"
    assert requests.get(f"http://127.0.0.1:{PORT}/nothing_here", timeout=10).status_code == 404
    serve.delete("app_a")
    r = requests.get(f"http://127.0.0.1:{PORT}/a", timeout=10)
    assert r.status_code == 404
    assert "app_a" not in serve.status()
    serve.delete("app_b")


def test_get_app_handle_and_deployment_handle(cluster):
    @serve.deployment
    class Echo:
        def __call__(self, x):
            return x

        def twice(self, x):
            return 2 * x

    serve.run(Echo.bind(), name="echo", route_prefix=None)
    h = serve.get_app_handle("echo")
    assert h.remote("hi").result() == "hi"
    assert h.twice.remote(4).result() == 8
    hd = serve.get_deployment_handle("Echo", app_name="echo")
    assert hd.options(method_name="twice").remote(5).result() == 10
    serve.delete("echo")


def test_handle_response_passed_to_another_call(cluster):
    @serve.deployment
    class Add:
        def __call__(self, x):
            return x + 1

    @serve.deployment
    class Outer:
        def __init__(self, add):
            self.add = add

        async def __call__(self, x):
            r1 = self.add.remote(x)
            r2 = self.add.remote(r1)  # a DeploymentResponse as an argument is resolved
            return await r2

    h = serve.run(Outer.bind(Add.bind()), name="chain", route_prefix=None)
    assert h.remote(1).result() == 3
    serve.delete("chain")


def test_model_multiplexing_routes_by_model_id(cluster):
    @serve.deployment(num_replicas=2)
    class M:
        @serve.multiplexed(max_num_models_per_replica=2)
        async def load(self, model_id: str):
            return {"id": model_id}

        async def __call__(self, x):
            mid = serve.get_multiplexed_model_id()
            m = await self.load(mid)
            import os

            return m["id"], os.getpid()

    h = serve.run(M.bind(), name="mux", route_prefix=None)
    outs = [h.options(multiplexed_model_id="m1").remote(0).result() for _ in range(8)]
    assert {o[0] for o in outs} == {"m1"}
    assert len({o[1] for o in outs}) == 1  # sticky to the replica that holds the model
    serve.delete("mux")


def test_retried_request_keeps_its_slot_until_the_reply(monkeypatch):
    """A request whose replica died is re-sent; the retried request's
    max_ongoing_requests slot must stay claimed while its reply is awaited (the dead
    replica's slot is returned immediately)."""
    import threading

    from ray_amd.exceptions import RayActorError
    from ray_amd.serve import handle as H

    class _Router:
        def __init__(self):
            self.lock = threading.Lock()
            self.done = []

        def _done_locked(self, rid):
            self.done.append(rid)

        def refresh(self, force=False):
            pass

        def mark_dead(self, rid):  # the failed replica leaves this handle's routing
            self.dead = rid

    router = _Router()
    s1, s2 = H._Slot(router, "dead"), H._Slot(router, "retry")
    seen = {}

    def fake_get(ref, timeout=None):
        if ref == "ref1":
            raise RayActorError("x", "replica died")
        seen["released_while_waiting"] = list(router.done)
        return 42

    monkeypatch.setattr(H.ray, "get", fake_get)
    retry = H.DeploymentResponse("ref2", router, slot=s2)
    resp = H.DeploymentResponse("ref1", router, slot=s1, resend=lambda: retry)
    assert resp.result() == 42
    assert seen["released_while_waiting"] == ["dead"]
    assert router.done == ["dead", "retry"] and router.dead == "dead"
