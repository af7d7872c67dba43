"""GCS durability (reference: src/ray/gcs/gcs_server/gcs_server.cc + gcs_table_storage:
GCS fault tolerance on an external store): with RAY_AMD_GCS_STORAGE_PATH the head raylet
persists its KV, job table, detached actors and detached placement groups, and a restarted
head reloads them — detached actors with restarts left come back (re-created, one more
restart; one with max_restarts exhausted stays dead), named PGs are re-placed, and the
previous head's running jobs are marked FAILED. The snapshot is written by a background
writer thread, off the head's control loop."""
import os
import time

import pytest

import ray_amd as ray
from ray_amd.experimental import internal_kv
from ray_amd.util.placement_group import get_placement_group, placement_group


@ray.remote
class Counter:
    def __init__(self, start=0):
        self.n = start

    def inc(self):
        self.n += 1
        return self.n


@pytest.fixture
def gcs_dir(tmp_path, monkeypatch):
    d = tmp_path / "gcs"
    monkeypatch.setenv("RAY_AMD_GCS_STORAGE_PATH", str(d))
    yield d
    if ray.is_initialized():
        ray.shutdown()


def test_head_restart_recovers_tables(gcs_dir):
    ray.init(num_cpus=4, namespace="durable")
    internal_kv._internal_kv_put(b"model_path", b"/ckpt/42", namespace="app")
    c = Counter.options(name="ctr", namespace="svc", lifetime="detached",
                        max_restarts=1).remote(10)
    assert ray.get(c.inc.remote()) == 11
    once = Counter.options(name="once", namespace="svc", lifetime="detached").remote()
    ray.get(once.inc.remote())  # max_restarts=0: the head restart is its one death
    tmp = Counter.remote()  # non-detached: dies with its job, not restored
    ray.get(tmp.inc.remote())
    pg = placement_group([{"CPU": 1}], name="pg_keep", lifetime="detached")
    assert pg.wait(10)
    time.sleep(0.6)  # the snapshot is written within 0.2 s of a change
    assert (gcs_dir / "gcs_snapshot.pkl").exists()
    ray.shutdown()

    ray.init(num_cpus=4, namespace="durable")  # a new head on the same storage
    from ray_amd._private.worker import _check_connected

    st = _check_connected().call_raylet("gcs_status")
    assert st["restored"]["actors"] == 2 and st["restored"]["pgs"] == 1
    assert internal_kv._internal_kv_get(b"model_path", namespace="app") == b"/ckpt/42"
    c2 = ray.get_actor("ctr", namespace="svc")
    assert ray.get(c2.inc.remote()) == 11  # re-created from its creation spec
    from ray_amd.util.state import list_actors, list_jobs

    acts = [a for a in list_actors() if a["name"] == "ctr"]
    assert acts and acts[0]["num_restarts"] >= 1
    with pytest.raises(ValueError):
        ray.get_actor("once", namespace="svc")
    dead = [a for a in list_actors() if a["name"] == "once"]
    assert dead and dead[0]["state"] == "DEAD"
    pg2 = get_placement_group("pg_keep")
    assert pg2.wait(10)
    jobs = list_jobs()
    assert any(j.get("status") in ("FAILED", "SUCCEEDED") for j in jobs if
               str(j.get("job_id")) != str(ray.get_runtime_context().get_job_id()))
    ray.kill(c2)
    ray.shutdown()


def test_without_storage_nothing_persists(tmp_path, monkeypatch):
    monkeypatch.delenv("RAY_AMD_GCS_STORAGE_PATH", raising=False)
    ray.init(num_cpus=2)
    internal_kv._internal_kv_put(b"k", b"v", namespace="x")
    ray.shutdown()
    ray.init(num_cpus=2)
    assert internal_kv._internal_kv_get(b"k", namespace="x") is None
    ray.shutdown()
