"""Memory monitor + worker-killing policy (modelled on python/ray/tests/
test_memory_pressure.py and src/ray/raylet/worker_killing_policy_*_test.cc).

Memory pressure is driven deterministically through a fake cgroup-v2 directory
(RAY_AMD_CGROUP_ROOT): the 'hog' task raises memory.current itself, exactly as a real
allocation would, and the raylet's monitor must kill it and let the owner retry."""

import os
import time

import pytest

import ray_amd as ray
from ray_amd._native import _core
from ray_amd._private.raylet import Lease, select_worker_to_kill
from ray_amd.exceptions import OutOfMemoryError, RayActorError


def _cg(tmp, limit, current, inactive=0):
    (tmp / "memory.max").write_text(f"{limit}\n")
    (tmp / "memory.current").write_text(f"{current}\n")
    (tmp / "memory.stat").write_text(f"anon {current}\ninactive_file {inactive}\n")


def test_monitor_reads_cgroup_and_threshold(tmp_path):
    _cg(tmp_path, 1000, 600, inactive=100)
    m = _core.MemoryMonitor(0.4, -1, str(tmp_path), "/proc")
    used, total, src = m.snapshot()
    assert (used, total, src) == (500, 1000, "cgroup2")
    assert m.over_threshold(used, total)
    # min_free_bytes relaxes the limit on big hosts: limit = max(0.4*1000, 1000-450)
    m2 = _core.MemoryMonitor(0.4, 450, str(tmp_path), "/proc")
    assert not m2.over_threshold(500, 1000)
    assert m.process_private_bytes(os.getpid()) > 0
    # no cgroup limit -> /proc/meminfo
    _, total2, src2 = _core.MemoryMonitor(0.95, -1, str(tmp_path / "none"), "/proc").snapshot()
    assert src2 == "meminfo" and total2 > 0


def _lease(owner, retriable, t):
    l = Lease(0, None, None, {}, owner, None, retriable)
    l.granted_at = t
    return l


def test_killing_policies():
    a1, a2, b1 = _lease("A", True, 1), _lease("A", True, 5), _lease("B", True, 9)
    nr = _lease("C", False, 20)
    # group_by_owner: largest retriable group (A), newest member of it
    v, retry = select_worker_to_kill([a1, a2, b1, nr], "group_by_owner")
    assert v is a2 and retry
    # a lone retriable lease is killed but not retried by the policy's hint
    v, retry = select_worker_to_kill([b1, nr], "group_by_owner")
    assert v is b1 and not retry
    # only non-retriable work left
    v, retry = select_worker_to_kill([nr], "group_by_owner")
    assert v is nr and not retry
    # retriable_fifo: retriable first, oldest first
    v, _ = select_worker_to_kill([nr, b1, a2, a1], "retriable_fifo")
    assert v is a1
    assert select_worker_to_kill([], "group_by_owner") == (None, False)


@pytest.fixture
def pressured(tmp_path, monkeypatch):
    _cg(tmp_path, 1 << 30, 100 << 20)
    monkeypatch.setenv("RAY_AMD_CGROUP_ROOT", str(tmp_path))
    monkeypatch.setenv("RAY_memory_usage_threshold", "0.5")
    monkeypatch.setenv("RAY_memory_monitor_refresh_ms", "50")
    ray.init(num_cpus=2)
    yield tmp_path
    ray.shutdown()


@pytest.fixture
def pressured_fifo(tmp_path, monkeypatch):
    monkeypatch.setenv("RAY_worker_killing_policy", "retriable_fifo")
    _cg(tmp_path, 1 << 30, 100 << 20)
    monkeypatch.setenv("RAY_AMD_CGROUP_ROOT", str(tmp_path))
    monkeypatch.setenv("RAY_memory_usage_threshold", "0.5")
    monkeypatch.setenv("RAY_memory_monitor_refresh_ms", "50")
    ray.init(num_cpus=2)
    yield tmp_path
    ray.shutdown()


def test_oom_kill_then_retry_succeeds(pressured_fifo):
    """retriable_fifo retries a killed retriable task (reference
    worker_killing_policy_retriable_fifo.cc: should_retry = the victim is retriable)."""
    cg = str(pressured_fifo)

    @ray.remote(max_retries=2)
    def hog(cg):
        marker = os.path.join(cg, "attempted")
        if not os.path.exists(marker):
            open(marker, "w").close()
            with open(os.path.join(cg, "memory.current"), "w") as f:
                f.write(f"{900 << 20}\n")  # "allocate" 900 MB of the 1 GB limit
            time.sleep(60)
            return "not killed"
        with open(os.path.join(cg, "memory.current"), "w") as f:
            f.write(f"{100 << 20}\n")
        return "ok after OOM retry"

    assert ray.get(hog.remote(cg), timeout=60) == "ok after OOM retry"


def test_oom_kill_lone_task_not_retried_by_group_by_owner(pressured):
    """group_by_owner does not retry the last task of its owner group (reference
    worker_killing_policy_group_by_owner.cc:87): the task fails with OutOfMemoryError even
    though it has retries left, instead of being re-killed until they run out."""
    cg = str(pressured)

    @ray.remote(max_retries=3)
    def hog(cg):
        marker = os.path.join(cg, "attempts")
        with open(marker, "a") as f:
            f.write("x")
        with open(os.path.join(cg, "memory.current"), "w") as f:
            f.write(f"{900 << 20}\n")
        time.sleep(60)

    with pytest.raises(OutOfMemoryError, match="low on memory"):
        ray.get(hog.remote(cg), timeout=60)
    with open(os.path.join(cg, "attempts")) as f:
        assert f.read() == "x"  # killed once, not retried
    with open(os.path.join(cg, "memory.current"), "w") as f:
        f.write(f"{100 << 20}\n")


def test_oom_kill_non_retriable_raises_out_of_memory(pressured):
    cg = str(pressured)

    @ray.remote(max_retries=0)
    def hog(cg):
        with open(os.path.join(cg, "memory.current"), "w") as f:
            f.write(f"{950 << 20}\n")
        time.sleep(60)

    with pytest.raises(OutOfMemoryError, match="low on memory"):
        ray.get(hog.remote(cg), timeout=60)
    with open(os.path.join(cg, "memory.current"), "w") as f:
        f.write(f"{100 << 20}\n")


def test_oom_kill_actor_reports_cause(pressured):
    cg = str(pressured)

    @ray.remote(max_restarts=0)
    class Hog:
        def eat(self, cg):
            with open(os.path.join(cg, "memory.current"), "w") as f:
                f.write(f"{990 << 20}\n")
            time.sleep(60)

    h = Hog.remote()
    with pytest.raises(RayActorError, match="out of memory"):
        ray.get(h.eat.remote(cg), timeout=60)
    with open(os.path.join(cg, "memory.current"), "w") as f:
        f.write(f"{100 << 20}\n")
