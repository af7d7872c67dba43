"""Runtime env, placement groups, state API, cancel and worker-reuse semantics (modelled on
python/ray/tests/test_runtime_env*.py, test_placement_group*.py, test_state_api.py,
test_cancel.py, test_worker_capping.py / test_basic_4.py)."""

import os
import time

import pytest

import ray_amd as ray
from ray_amd.util.placement_group import (placement_group, placement_group_table,
                                          remove_placement_group)
from ray_amd.util.scheduling_strategies import PlacementGroupSchedulingStrategy


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_runtime_env_per_task_and_per_actor(cluster):
    @ray.remote
    def env(k):
        return os.environ.get(k)

    assert ray.get(env.options(runtime_env={"env_vars": {"RA_X": "1"}}).remote("RA_X")) == "1"
    assert ray.get(env.remote("RA_X")) is None  # not leaked into other workers' tasks

    @ray.remote
    class A:
        def get(self, k):
            return os.environ.get(k)

    a = A.options(runtime_env={"env_vars": {"RA_Y": "yes"}}).remote()
    assert ray.get(a.get.remote("RA_Y")) == "yes"


def test_runtime_env_working_dir_module_import(cluster, tmp_path):
    d = tmp_path / "wd"
    d.mkdir()
    (d / "helper_mod_ra.py").write_text("VALUE = 41\n")

    @ray.remote
    def use():
        import helper_mod_ra

        return helper_mod_ra.VALUE + 1

    assert ray.get(use.options(runtime_env={"working_dir": str(d)}).remote()) == 42


def test_pg_bundle_resources_are_reserved(cluster):
    pg = placement_group([{"CPU": 2}], strategy="PACK")
    assert pg.wait(10)
    avail = ray.available_resources().get("CPU", 0)
    assert avail <= 2 + 1e-6

    @ray.remote(num_cpus=2)
    def inside():
        return "ok"

    ref = inside.options(scheduling_strategy=PlacementGroupSchedulingStrategy(pg)).remote()
    assert ray.get(ref, timeout=20) == "ok"
    table = placement_group_table(pg)
    assert table["state"] == "CREATED" and table["bundles"][0]["CPU"] == 2
    remove_placement_group(pg)
    time.sleep(0.3)
    assert ray.available_resources().get("CPU", 0) >= 4 - 1e-6


def test_pg_removal_kills_its_actors(cluster):
    pg = placement_group([{"CPU": 1}])
    assert pg.wait(10)

    @ray.remote(num_cpus=1)
    class Pinned:
        def ping(self):
            return 1

    a = Pinned.options(scheduling_strategy=PlacementGroupSchedulingStrategy(pg)).remote()
    assert ray.get(a.ping.remote()) == 1
    remove_placement_group(pg)
    with pytest.raises(ray.exceptions.RayActorError):
        for _ in range(100):
            ray.get(a.ping.remote(), timeout=5)
            time.sleep(0.05)


def test_cancel_running_task_and_queued_task(cluster):
    @ray.remote
    def spin():
        while True:
            time.sleep(0.01)

    r = spin.remote()
    time.sleep(0.3)
    ray.cancel(r, force=True)
    with pytest.raises((ray.exceptions.TaskCancelledError, ray.exceptions.WorkerCrashedError,
                        ray.exceptions.RayTaskError)):
        ray.get(r, timeout=20)

    @ray.remote(num_cpus=4)
    def hog():
        time.sleep(2)
        return 1

    h = hog.remote()
    queued = hog.remote()  # waits for the CPUs the first one holds
    ray.cancel(queued)
    with pytest.raises(ray.exceptions.TaskCancelledError):
        ray.get(queued, timeout=20)
    assert ray.get(h, timeout=20) == 1


def test_state_api_reflects_lifecycle(cluster):
    from ray_amd.util.state import list_actors, list_tasks

    @ray.remote
    class Named:
        def ping(self):
            return 1

    a = Named.options(name="state_probe").remote()
    ray.get(a.ping.remote())
    acts = [x for x in list_actors() if x.get("name") == "state_probe"]
    assert acts and acts[0]["state"] == "ALIVE"
    ray.kill(a)
    time.sleep(0.5)
    acts = [x for x in list_actors() if x.get("name") == "state_probe"]
    assert acts and acts[0]["state"] == "DEAD"

    @ray.remote
    def tagged():
        return 1

    ray.get([tagged.remote() for _ in range(3)])
    time.sleep(1.5)  # task events are flushed periodically
    done = [t for t in list_tasks() if "tagged" in (t.get("name") or "")]
    assert len(done) >= 3 and all(t["state"] in ("FINISHED", "RUNNING") for t in done)


def test_worker_processes_are_reused(cluster):
    @ray.remote
    def pid():
        return os.getpid()

    pids = set(ray.get([pid.remote() for _ in range(40)]))
    assert len(pids) <= 4 + 1  # bounded by the CPU slots, not one process per task


def test_available_resources_restored_after_actor_death(cluster):
    for _ in range(50):  # idle worker leases of earlier tests are returned asynchronously
        if ray.available_resources().get("CPU", 0) >= 4 - 1e-6:
            break
        time.sleep(0.1)
    before = ray.available_resources().get("CPU", 0)

    @ray.remote(num_cpus=2)
    class Big:
        def ping(self):
            return 1

    b = Big.remote()
    ray.get(b.ping.remote())
    assert ray.available_resources().get("CPU", 0) <= before - 2 + 1e-6
    ray.kill(b)
    for _ in range(50):
        if ray.available_resources().get("CPU", 0) >= before - 1e-6:
            break
        time.sleep(0.1)
    assert ray.available_resources().get("CPU", 0) >= before - 1e-6
