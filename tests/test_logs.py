"""Per-worker log files + state list_logs / get_log (reference: python/ray/tests/
test_state_api_log.py)."""

import os
import time

import pytest

import ray_amd as ray
from ray_amd.util.state import get_log, list_logs


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=2)
    yield
    ray.shutdown()


def test_worker_logs_captured(cluster):
    @ray.remote
    class Talker:
        def say(self, msg):
            print(msg, flush=True)
            import sys

            print("ERR " + msg, file=sys.stderr, flush=True)
            return os.getpid()

    a = Talker.remote()
    pid = ray.get(a.say.remote("hello-from-actor"))
    deadline = time.time() + 10
    lines = []
    while time.time() < deadline:
        try:
            lines = list(get_log(pid=pid))
        except FileNotFoundError:
            lines = []
        if any("hello-from-actor" in ln for ln in lines):
            break
        time.sleep(0.2)
    assert any("hello-from-actor" in ln for ln in lines)
    errs = []
    while time.time() < deadline + 5:  # stderr is pumped by its own thread
        errs = list(get_log(pid=pid, suffix="err"))
        if any("ERR hello-from-actor" in ln for ln in errs):
            break
        time.sleep(0.1)
    assert any("ERR hello-from-actor" in ln for ln in errs)
    logs = list_logs()
    assert any(str(pid) in f for f in logs["worker_out"])
    assert list(get_log(pid=pid, tail=1))[-1] == lines[-1]
