"""Serve replica failure: a replica killed while requests are in flight — the handle retries
those requests on a live replica, the controller's health check notices the death and
starts a replacement, and the application is back at its target replica count (modelled on
python/ray/serve/tests/test_failure.py)."""

import time

import pytest

import ray_amd as ray
from ray_amd import serve
from ray_amd.serve._controller import CONTROLLER_NAME, SERVE_NAMESPACE


def _wait_for(cond, timeout=30, msg="condition not met"):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if cond():
            return
        time.sleep(0.05)
    raise AssertionError(msg)


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=6)
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    serve.start(http_options={"port": port})
    yield
    serve.shutdown()
    ray.shutdown()


def test_replica_killed_mid_request_is_retried_and_replaced(cluster):
    @serve.deployment(num_replicas=2, health_check_period_s=0.2, health_check_timeout_s=2.0)
    class Slow:
        def __call__(self, x):
            import os

            time.sleep(0.5)
            return os.getpid(), x

    h = serve.run(Slow.bind(), name="ft", route_prefix="/ft")
    pids = {h.remote(i).result()[0] for i in range(8)}
    assert len(pids) == 2
    ctrl = ray.get_actor(CONTROLLER_NAME, namespace=SERVE_NAMESPACE)
    before = ray.get(ctrl.get_replicas.remote("ft", "Slow"))[1]  # [(replica id, actor)]
    resps = [h.remote(i) for i in range(6)]  # spread over both replicas
    time.sleep(0.15)
    victim_id, actor = before[0]
    ray.kill(actor)
    # every in-flight request completes, the killed replica's share on the survivor
    out = [r.result(timeout_s=30) for r in resps]
    assert sorted(x for _, x in out) == list(range(6))
    # the controller replaces the dead replica; the app returns to 2 live replicas
    _wait_for(lambda: serve.status()["ft"]["deployments"]["Slow"]["replica_states"].get(
        "RUNNING", 0) == 2 and len({h.remote(i).result()[0] for i in range(10)}) == 2,
        timeout=40, msg="dead replica was not replaced")
    after = [rid for rid, _ in ray.get(ctrl.get_replicas.remote("ft", "Slow"))[1]]
    assert victim_id not in after and len(after) == 2
    serve.delete("ft")


def test_deployment_options_validated_and_graceful_wait_loop(cluster):
    with pytest.raises(TypeError, match="unsupported deployment option"):
        serve.deployment(lambda: 1, no_such_option=3)
    with pytest.raises(ValueError):
        serve.deployment(lambda: 1, logging_config={"log_level": "LOUD"})

    @serve.deployment(graceful_shutdown_wait_loop_s=0.05, graceful_shutdown_timeout_s=10,
                      logging_config={"log_level": "DEBUG", "enable_access_log": True})
    class Busy:
        def __call__(self, t):
            import logging

            time.sleep(t)
            return logging.getLogger().getEffectiveLevel()

    h = serve.run(Busy.bind(), name="gw", route_prefix="/gw")
    import logging

    assert h.remote(0).result() == logging.DEBUG  # the replica applied logging_config
    slow = h.remote(1.0)
    time.sleep(0.2)
    t0 = time.time()
    serve.delete("gw")  # drains: the in-flight request still completes
    assert slow.result(timeout_s=15) == logging.DEBUG
    assert time.time() - t0 < 10
