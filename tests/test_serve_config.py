"""Serve backpressure, declarative config files and the serve CLI (modelled on
python/ray/serve/tests/test_max_queued_requests.py, test_deploy_app.py, test_cli.py,
unit/test_schema.py)."""

import asyncio
import os
import pathlib
import shutil
import socket
import subprocess
import sys
import tempfile
import textwrap
import time

import pytest
import requests

import ray_amd as ray
from ray_amd import serve
from ray_amd.serve.exceptions import BackPressureError

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PORT = 18177


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@ray.remote(num_cpus=0)
class Signal:
    def __init__(self):
        self.ev = asyncio.Event()
        self.waiters = 0

    async def wait(self):
        self.waiters += 1
        await self.ev.wait()
        self.waiters -= 1

    def send(self):
        self.ev.set()

    def num_waiters(self):
        return self.waiters


def _wait_for(cond, timeout=20):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if cond():
            return
        time.sleep(0.05)
    raise AssertionError("condition not met")


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=8)
    serve.start(http_options={"port": PORT})
    yield
    serve.shutdown()
    ray.shutdown()


def test_handle_backpressure(cluster):
    sig = Signal.remote()

    @serve.deployment(max_ongoing_requests=1, max_queued_requests=1)
    class D:
        async def __call__(self, msg):
            await sig.wait.remote()
            return msg

    h = serve.run(D.bind(), name="bp", route_prefix=None)
    first = h.remote("hi-1")
    _wait_for(lambda: ray.get(sig.num_waiters.remote()) == 1)
    second = h.remote("hi-2")  # queued at the handle: .remote() itself does not block
    for _ in range(5):
        with pytest.raises(BackPressureError) as ei:
            h.remote("dropped").result()
        assert ei.value.message.startswith("Request dropped due to backpressure")
    ray.get(sig.send.remote())
    assert first.result(timeout_s=20) == "hi-1"
    assert second.result(timeout_s=20) == "hi-2"
    serve.delete("bp")


def test_http_backpressure_503(cluster):
    sig = Signal.remote()

    @serve.deployment(max_ongoing_requests=1, max_queued_requests=1)
    class D:
        async def __call__(self, request):
            await sig.wait.remote()
            return "ok"

    serve.run(D.bind(), name="bphttp", route_prefix="/bp")

    @ray.remote(num_cpus=0)
    def get():
        r = requests.get(f"http://127.0.0.1:{PORT}/bp", timeout=60)
        return r.status_code, r.text

    first = get.remote()
    _wait_for(lambda: ray.get(sig.num_waiters.remote()) == 1)
    second = get.remote()
    time.sleep(0.5)  # let the second request reach the proxy's queue
    for _ in range(3):
        code, text = ray.get(get.remote())
        assert code == 503 and text.startswith("Request dropped due to backpressure")
    ray.get(sig.send.remote())
    assert ray.get(first) == (200, "ok")
    assert ray.get(second) == (200, "ok")
    serve.delete("bphttp")


def test_max_ongoing_requests_caps_replica_concurrency(cluster):
    @serve.deployment(max_ongoing_requests=2)
    class C:
        def __init__(self):
            self.cur = 0
            self.peak = 0

        async def __call__(self):
            self.cur += 1
            self.peak = max(self.peak, self.cur)
            await asyncio.sleep(0.2)
            self.cur -= 1
            return self.peak

    h = serve.run(C.bind(), name="cap", route_prefix=None)
    resps = [h.remote() for _ in range(8)]  # returns at once; 6 wait at the handle
    peaks = [r.result(timeout_s=30) for r in resps]
    assert max(peaks) == 2
    # fire-and-forget requests release their slots when the reply lands
    for _ in range(4):
        h.remote()
    time.sleep(1.0)
    t0 = time.time()
    assert h.remote().result(timeout_s=10) == 2
    assert time.time() - t0 < 2.0
    serve.delete("cap")


def test_autoscaling_config_model_validation():
    from ray_amd.serve.config import AutoscalingConfig, normalize_autoscaling_config

    with pytest.raises(ValueError):
        AutoscalingConfig(min_replicas=3, max_replicas=2)
    with pytest.raises(ValueError):
        AutoscalingConfig(min_replicas=1, max_replicas=4, initial_replicas=5)
    d = normalize_autoscaling_config(AutoscalingConfig(min_replicas=1, max_replicas=4,
                                                       target_ongoing_requests=3))
    assert d["target_ongoing_requests"] == 3 and d["max_replicas"] == 4
    with pytest.raises(ValueError):
        normalize_autoscaling_config({"min_replicas": 1, "bogus": 2})
    # deprecated alias maps onto the target
    d = normalize_autoscaling_config({"target_num_ongoing_requests_per_replica": 5,
                                      "max_replicas": 2})
    assert d["target_ongoing_requests"] == 5


def test_schema_validation():
    from ray_amd.serve.schema import DeploymentSchema, ServeDeploySchema

    with pytest.raises(ValueError):
        ServeDeploySchema(applications=[{"name": "a", "import_path": "m:x"},
                                        {"name": "a", "import_path": "m:y",
                                         "route_prefix": "/y"}])
    with pytest.raises(ValueError):
        ServeDeploySchema(applications=[{"name": "a", "import_path": "m:x"},
                                        {"name": "b", "import_path": "m:y"}])  # both at "/"
    with pytest.raises(ValueError):
        ServeDeploySchema(applications=[{"import_path": "m:x", "route_prefix": "nope"}])
    with pytest.raises(ValueError):
        DeploymentSchema(name="d", num_replicas=2, autoscaling_config={"max_replicas": 3})
    assert DeploymentSchema(name="d", num_replicas=3).overrides() == {"num_replicas": 3}


APP_MODULE = textwrap.dedent('''
    from pydantic import BaseModel

    from ray_amd import serve


    @serve.deployment
    class Greeter:
        def __init__(self, greeting="hello"):
            self.greeting = greeting
            self.suffix = ""

        def reconfigure(self, cfg):
            self.suffix = cfg.get("suffix", "")

        def __call__(self, name):
            return f"{self.greeting} {name}{self.suffix}"


    @serve.deployment
    class Ingress:
        def __init__(self, greeter):
            self.greeter = greeter

        async def __call__(self, request):
            name = request.query_params.get("name", "world")
            return await self.greeter.remote(name)


    class Args(BaseModel):
        greeting: str = "hello"


    def builder(args: Args):
        return Ingress.bind(Greeter.bind(args.greeting))


    app = Ingress.bind(Greeter.bind())
''')


@pytest.fixture()
def app_dir():
    d = pathlib.Path(tempfile.mkdtemp(prefix="serveapp"))
    (d / "greet_app.py").write_text(APP_MODULE)
    yield d
    shutil.rmtree(d, ignore_errors=True)
    sys.modules.pop("greet_app", None)


def test_deploy_config_builder_overrides_and_declarative_delete(cluster, app_dir):
    from ray_amd.serve.schema import deploy_config, get_deployed_config

    cfg = {
        "http_options": {"port": PORT},
        "applications": [
            {"name": "greet", "route_prefix": "/greet", "import_path": "greet_app:builder",
             "args": {"greeting": "hey"}, "runtime_env": {"working_dir": str(app_dir)},
             "deployments": [{"name": "Greeter", "num_replicas": 2,
                              "user_config": {"suffix": "!"}}]},
            {"name": "plain", "route_prefix": "/plain", "import_path": "greet_app.app",
             "runtime_env": {"working_dir": str(app_dir)}},
        ],
    }
    deploy_config(cfg)
    r = requests.get(f"http://127.0.0.1:{PORT}/greet", params={"name": "amd"}, timeout=30)
    assert r.status_code == 200 and r.text == "hey amd!", r.text
    r = requests.get(f"http://127.0.0.1:{PORT}/plain", timeout=30)
    assert r.text == "hello world"
    st = serve.status()
    assert st["greet"]["deployments"]["Greeter"]["replica_states"]["RUNNING"] == 2
    assert get_deployed_config()["applications"][0]["args"] == {"greeting": "hey"}
    # declarative: an app left out of the next config is deleted
    cfg["applications"] = cfg["applications"][:1]
    cfg["applications"][0]["deployments"][0]["user_config"] = {"suffix": "?"}
    deploy_config(cfg)
    assert "plain" not in serve.status()
    _wait_for(lambda: requests.get(f"http://127.0.0.1:{PORT}/greet", timeout=30).text ==
              "hey world?")
    assert requests.get(f"http://127.0.0.1:{PORT}/plain", timeout=30).status_code == 404
    serve.delete("greet")


def test_deploy_config_rejects_unknown_deployment(cluster, app_dir):
    from ray_amd.serve.schema import deploy_config

    with pytest.raises(ValueError, match="Nope"):
        deploy_config({"applications": [{
            "name": "bad", "route_prefix": "/bad", "import_path": "greet_app.app",
            "runtime_env": {"working_dir": str(app_dir)},
            "deployments": [{"name": "Nope", "num_replicas": 1}]}]})


def test_serve_cli_build_deploy_status_config_shutdown(app_dir):
    tmp = pathlib.Path(tempfile.mkdtemp(prefix="sc", dir="/tmp"))  # short: unix sockets
    env = dict(os.environ, RAY_AMD_TMPDIR=str(tmp), PYTHONPATH=REPO)
    env.pop("RAY_ADDRESS", None)
    port = _free_port()

    def run(mod, *args, timeout=180):
        return subprocess.run([sys.executable, "-m", mod, *args], env=env, cwd=str(app_dir),
                              capture_output=True, text=True, timeout=timeout,
                              stdin=subprocess.DEVNULL)

    import yaml

    r = run("ray_amd.serve", "build", "greet_app:app", "-o", "cfg.yaml")
    assert r.returncode == 0, r.stderr
    cfg = yaml.safe_load((app_dir / "cfg.yaml").read_text())
    names = [d["name"] for d in cfg["applications"][0]["deployments"]]
    assert names == ["Greeter", "Ingress"]
    cfg["http_options"] = {"port": port}
    cfg["applications"][0]["deployments"][0]["num_replicas"] = 2
    (app_dir / "cfg.yaml").write_text(yaml.safe_dump(cfg))

    dash = _free_port()
    r = run("ray_amd.scripts", "start", "--head", "--num-cpus", "4", "--dashboard-port",
            str(dash))
    assert r.returncode == 0, r.stderr
    try:
        r = run("ray_amd.serve", "deploy", "cfg.yaml")
        assert r.returncode == 0, r.stdout + r.stderr
        resp = requests.get(f"http://127.0.0.1:{port}/", params={"name": "cli"}, timeout=30)
        assert resp.text == "hello cli"
        r = run("ray_amd.serve", "status")
        st = yaml.safe_load(r.stdout)["applications"]["default"]
        assert st["status"] == "RUNNING"
        assert st["deployments"]["Greeter"]["replica_states"]["RUNNING"] == 2
        r = run("ray_amd.serve", "config")
        assert yaml.safe_load(r.stdout)["import_path"] == "greet_app:app"
        # the same through the dashboard's Serve REST API (/api/serve/applications/)
        url = f"http://127.0.0.1:{dash}"
        r = run("ray_amd.serve", "status", "--address", url)
        assert r.returncode == 0, r.stderr
        st = yaml.safe_load(r.stdout)["applications"]["default"]
        assert st["status"] == "RUNNING"
        r = run("ray_amd.serve", "config", "--address", url)
        assert yaml.safe_load(r.stdout)["import_path"] == "greet_app:app"
        cfg["applications"][0]["deployments"][0]["num_replicas"] = 1
        cfg["applications"][0]["deployments"][0]["user_config"] = {"suffix": "!"}
        (app_dir / "cfg.yaml").write_text(yaml.safe_dump(cfg))
        r = run("ray_amd.serve", "deploy", "cfg.yaml", "--address", url)
        assert r.returncode == 0, r.stdout + r.stderr
        _wait_for(lambda: requests.get(f"http://127.0.0.1:{port}/", params={"name": "rest"},
                                       timeout=30).text == "hello rest!")
        r = run("ray_amd.serve", "shutdown", "-y", "--address", url)
        assert r.returncode == 0, r.stderr
        r = run("ray_amd.serve", "status")
        assert yaml.safe_load(r.stdout)["applications"] == {}
    finally:
        run("ray_amd.scripts", "stop")
        shutil.rmtree(tmp, ignore_errors=True)


def test_replica_context_and_serve_metrics(cluster):
    import pickle

    from ray_amd.serve import metrics as smetrics
    from ray_amd.serve.exceptions import RayServeException
    from ray_amd.util.metrics import prometheus_text

    with pytest.raises(RayServeException):
        serve.get_replica_context()

    @serve.deployment(num_replicas=2)
    class Ctx:
        def __init__(self):
            self.at_init = serve.get_replica_context().deployment  # visible in __init__
            self.hits = smetrics.Counter("serve_ctx_hits", "requests", tag_keys=("kind",))

        def __call__(self):
            rc = serve.get_replica_context()
            self.hits.inc(tags={"kind": "call"})
            assert rc.servable_object is self
            return rc.app_name, rc.deployment, rc.replica_tag, self.at_init, \
                rc.replica_id.unique_id

    h = serve.run(Ctx.bind(), name="ctxapp", route_prefix=None)
    outs = {h.remote().result() for _ in range(12)}
    assert {o[:2] for o in outs} == {("ctxapp", "Ctx")}
    assert all(o[3] == "Ctx" and o[2].endswith(o[4]) for o in outs)
    m = smetrics.Gauge("serve_test_gauge", tag_keys=("k",))
    assert pickle.loads(pickle.dumps(m))._tag_keys == m._tag_keys
    with pytest.raises(ValueError):
        smetrics.Counter("bad", tag_keys=("deployment",))
    serve.delete("ctxapp")
    prometheus_text()  # renders with the serve tag keys


def test_batch_streaming_and_runtime_retuning(cluster):
    @serve.deployment(max_ongoing_requests=32)
    class B:
        def __init__(self):
            self.sizes = []

        @serve.batch(max_batch_size=4, batch_wait_timeout_s=0.2)
        async def tokens(self, ns):
            self.sizes.append(len(ns))
            for step in range(max(ns)):
                yield [f"{n}:{step}" if step < n else None for n in ns]

        @serve.batch(max_batch_size=2, batch_wait_timeout_s=0.2)
        async def double(self, xs):
            self.sizes.append(len(xs))
            return [2 * x for x in xs]

        def retune(self, n):
            self.double.set_max_batch_size(n)
            self.double.set_batch_wait_timeout_s(0.3)
            return self.double._get_max_batch_size(), self.double._get_batch_wait_timeout_s()

        def sizes_seen(self):
            out, self.sizes = self.sizes, []
            return out

    h = serve.run(B.bind(), name="batchx", route_prefix=None)
    gens = [h.options(method_name="tokens", stream=True).remote(n) for n in (1, 2, 3)]
    streams = [list(g) for g in gens]
    assert streams[2][:3] == ["3:0", "3:1", "3:2"]
    assert streams[0][0] == "1:0" and streams[1][:2] == ["2:0", "2:1"]
    assert max(h.sizes_seen.remote().result()) > 1  # the three streams shared batches
    resps = [h.double.remote(i) for i in range(8)]
    assert [r.result() for r in resps] == [2 * i for i in range(8)]
    assert max(h.sizes_seen.remote().result()) <= 2
    assert h.retune.remote(8).result() == (8, 0.3)
    resps = [h.double.remote(i) for i in range(8)]
    assert [r.result() for r in resps] == [2 * i for i in range(8)]
    assert max(h.sizes_seen.remote().result()) > 2
    serve.delete("batchx")


def test_batch_decorator_validation():
    with pytest.raises(TypeError):
        @serve.batch
        def not_async(xs):
            return xs
    with pytest.raises(ValueError):
        serve.batch(max_batch_size=0)
